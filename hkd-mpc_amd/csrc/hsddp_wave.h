// hsddp_wave.h — wave-level building blocks of the one-wave-per-workgroup solver kernels (gfx950).
//
// DPP row broadcasts (row_newbcast), fused broadcast multiply-adds, the half-wave exchange, the
// f64 / f32 16x16x4 MFMA tile and small reductions.  Inline asm where the compiler has no
// builtin for the fused form; every VGPR a DPP instruction reads was written at least two VALU
// instructions earlier unless the caller asks for the s_nop (`fresh`).
#pragma once
#include <type_traits>
#include <utility>

#include "hsddp_device.h"

namespace hsddp {

// A one-wave workgroup's barrier is no instruction and stops no code motion; the memory clobber
// keeps each stage's LDS accesses in their stage.  LDS operations of one wave complete in order.
#define HSYNC()                        \
    do {                               \
        __syncthreads();               \
        asm volatile("" ::: "memory"); \
    } while (0)
#define LSYNC() asm volatile("" ::: "memory")

// Compile-time loop: the body sees its index as a constant, so register arrays indexed by it stay
// in VGPRs.
template <typename F, int... I>
DEV void static_for_impl(F &&f, std::integer_sequence<int, I...>)
{
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
DEV void static_for(F &&f)
{
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// a value known to be equal on all lanes, moved to SGPRs
DEV double uniform(double v)
{
    const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
    const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
    return __hiloint2double(hi, lo);
}
DEV float uniform(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }

// v on lane `src`, broadcast to every lane through SGPRs
DEV double lane_value(double v, int src)
{
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
    return __hiloint2double(hi, lo);
}
DEV float lane_value(float v, int src) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src)); }
DEV int lane_value(int v, int src) { return __builtin_amdgcn_readlane(v, src); }

// 1 / x from the hardware reciprocal refined by Newton steps (within an ulp of the quotient)
DEV double recip(double x)
{
    double r = __builtin_amdgcn_rcp(x);
    double e = __builtin_fma(-x, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-x, r, 1.0);
    return __builtin_fma(r, e, r);
}
DEV float recip(float x)
{
    float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(r, e, r);
}

// value held by the same lane of the other half-wave (call with all 64 lanes active; any wave of
// a multi-wave workgroup)
DEV double other_half(double v)
{
    const unsigned lo = __double2loint(v), hi = __double2hiint(v);
    const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    return (threadIdx.x & 32) == 0 ? __hiloint2double(b[1], a[1]) : __hiloint2double(b[0], a[0]);
}
DEV float other_half(float v)
{
    const unsigned u = __float_as_uint(v);
    const auto a = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    return __uint_as_float((threadIdx.x & 32) == 0 ? a[1] : a[0]);
}

// sum over the 32 lanes of this lane's half-wave (every lane of the half gets it)
template <typename real>
DEV real half_sum(real v)
{
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// v on lane j of this lane's 16-lane DPP row (row_newbcast; the s_nop gives a VGPR written by the
// previous VALU instruction its two wait states)
template <int j, typename T>
DEV T row_bcast(T v)
{
    T r;
    if constexpr (sizeof(T) == 8)
        asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(v), "i"(j));
    else
        asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(v), "i"(j));
    return r;
}

// w += (w on lane j of this lane's 16-lane row) * s; `fresh`: w may have been written by the
// instruction just before
template <int j, bool fresh, typename T>
DEV void fmac_row_bcast(T &w, T s)
{
    if constexpr (sizeof(T) == 8) {
        if constexpr (fresh)
            asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
                         : "+v"(w)
                         : "v"(s), "i"(j));
        else
            asm volatile("v_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "+v"(w) : "v"(s), "i"(j));
    } else {
        if constexpr (fresh)
            asm volatile("s_nop 1\n\tv_fmac_f32_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
                         : "+v"(w)
                         : "v"(s), "i"(j));
        else
            asm volatile("v_fmac_f32_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "+v"(w) : "v"(s), "i"(j));
    }
}

// acc += (coef on lane j of this lane's 16-lane DPP row) * x — a broadcast coefficient in the
// multiply-add itself.  coef must not have been written by the previous two VALU instructions.
template <int j, typename T>
DEV void bfma(T &acc, T coef, T x)
{
    if constexpr (sizeof(T) == 8)
        asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(coef), "v"(x), "i"(j));
    else
        asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(coef), "v"(x), "i"(j));
}

// DPP sources that VALU instructions produce (e.g. values converted to fp32): every value exists
// before the s_nop, which gives the last of them its two wait states before the first DPP read
// (the inline-asm DPP instructions are invisible to the compiler's hazard recognizer;
// tools/dpp_hazards.py checks the emitted code)
template <typename T, int N>
DEV void dpp_ready(T (&a)[N])
{
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "+v"(a[i]));
    asm volatile("s_nop 1");
}

// acc += V[n] * x, where the coefficient vector V is spread over the DPP row: V[16 k + j] is held
// by register cf[k] of position j (compile-time n)
template <int n, typename T, int NC>
DEV void vfma(T &acc, const T (&cf)[NC], T x)
{
    static_assert((n >> 4) < NC, "coefficient register");
    bfma<(n & 15)>(acc, cf[n >> 4], x);
}

// D = A B + C on a 16 x 16 x 4 MFMA tile (one operand value per lane: A[l & 15][l >> 4],
// B[l >> 4][l & 15]); result register g of lane l is row mfma_row(l >> 4, g), column l & 15 — the
// f64 form interleaves rows, the f32 form blocks them (cdna_hip_programming.md, fragment layout)
typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
DEV d4 mfma16(double a, double b, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }
DEV f4 mfma16(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
template <typename real> using acc4 = std::conditional_t<sizeof(real) == 8, d4, f4>;
template <typename real>
DEV constexpr int mfma_row(int lk, int g) { return sizeof(real) == 8 ? lk + 4 * g : 4 * lk + g; }

// One LDS-DMA instruction: 16 bytes per active lane from `src` to LDS at m0 + 16 * lane (inline
// asm: the compiler neither waits for it nor knows it writes LDS — the consumer waits with
// vmcnt).  M0 is compiler-reserved: saved, set with one wait state before the DMA, restored.
DEV void lds_dma16(const void *src, unsigned m0)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(m0)
                 : "memory");
}

// the same with the non-temporal policy (nt): for bytes this launch reads once and nothing reads
// again soon (tools/micro/lin_streams.hip: a 3.3 GB stream of knot images 6.2 -> 7.0 TB/s)
DEV void lds_dma16_nt(const void *src, unsigned m0)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(m0)
                 : "memory");
}

// LDS atomic add without return (ds_add_f64 / ds_add_f32): the IEEE round-to-nearest add of v to
// the stored value, queued behind the wave's earlier LDS operations
template <typename real>
DEV void lds_add(real *p, real v)
{
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

}  // namespace hsddp

namespace hsddp {

// The pivot chain's scalar operations (hsddp_sweep.hip, eliminate): the hardware reciprocal, the
// Newton step's two multiply-adds and the negated product.  Round 4 wrote them as inline asm, placed
// by hand between the (volatile, inline-asm) DPP multiply-adds; as builtins the compiler schedules
// them and, seeing what they are, inserts only the wait states they need (the knot's s_nop count
// 145 -> 89): the same instructions and results, C1 16.19 -> 16.0 ms, the sweep at B = 256
// 0.743 -> 0.724 ms, B = 4096 unchanged (A/B on one box, round 5).
DEV void asm_rcp(double &r, double x) { r = __builtin_amdgcn_rcp(x); }
DEV void asm_rcp(float &r, float x) { r = __builtin_amdgcn_rcpf(x); }
// e = 1 - x r
DEV void asm_nfma1(double &e, double x, double r) { e = __builtin_fma(-x, r, 1.0); }
DEV void asm_nfma1(float &e, float x, float r) { e = __builtin_fmaf(-x, r, 1.0f); }
// r = r + r e
DEV void asm_newton(double &r, double e) { r = __builtin_fma(r, e, r); }
DEV void asm_newton(float &r, float e) { r = __builtin_fmaf(r, e, r); }
// y = -(a b)
DEV void asm_nmul(double &y, double a, double b) { y = -(a * b); }
DEV void asm_nmul(float &y, float a, float b) { y = -(a * b); }


// The values of x on the two 16-lane DPP rows of this lane's half-wave, at this lane's DPP
// position: ka from the first row (lanes 0..15 / 32..47), kb from the second (v_permlane16_swap).
DEV void row_pair(double x, double &ka, double &kb)
{
    const unsigned lo = __double2loint(x), hi = __double2hiint(x);
    const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    ka = __hiloint2double(b[0], a[0]);
    kb = __hiloint2double(b[1], a[1]);
}
DEV void row_pair_last_f(float x, float &ka, float &kb)
{
    const unsigned u = __float_as_uint(x);
    const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    ka = __uint_as_float(a[0]);
    kb = __uint_as_float(a[1]);
}
// The same when x is not used afterwards: one 64-bit copy (x's own registers take the other
// result), not a copy per 32-bit half for each operand of the swaps
DEV void row_pair_last(double x, double &ka, double &kb)
{
    double c;
    asm volatile("v_mov_b64 %0, %1" : "=v"(c) : "v"(x));
    const auto a = __builtin_amdgcn_permlane16_swap(__double2loint(c), __double2loint(x), false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(__double2hiint(c), __double2hiint(x), false, false);
    ka = __hiloint2double(b[0], a[0]);
    kb = __hiloint2double(b[1], a[1]);
}
DEV void row_pair_last(float x, float &ka, float &kb) { row_pair_last_f(x, ka, kb); }
DEV void row_pair(float x, float &ka, float &kb)
{
    const unsigned u = __float_as_uint(x);
    const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    ka = __uint_as_float(a[0]);
    kb = __uint_as_float(a[1]);
}

}  // namespace hsddp
