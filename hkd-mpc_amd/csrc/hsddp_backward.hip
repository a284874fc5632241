// hsddp_backward.hip — regularised backward Riccati sweep + multiple-shooting linear rollout.
//
// MultiPhaseDDP::backward_sweep_regularized / backward_sweep / linear_rollout
//   (HSDDPSolver/source/MultiPhaseDDP.cpp:20-50, 141-229) over SinglePhase::backward_sweep /
//   linear_rollout (SinglePhase.cpp:144-178, 298-367), for B independent elements.
//
// k_riccati (gfx950): one 64-lane wave per element.  Lane L has row r = L & 31 and half
// hf = L >> 5; a row lane (r < 24) owns columns 12 hf .. 12 hf + 11 of row r of the value
// Hessian H, of Qxx, of Quu and of Qux^T — 12-double register arrays, so 4 waves/SIMD fit in
// the register file and the 4096 elements of the metric batch are all resident at once.
// Lane 24 of each half ("vector lane") owns that half of Qu.  The halves exchange values with
// v_permlane32_swap (VALU, no LDS round trip).  Values every lane reads at the same address
// (the knot's LQ record, phase constants) come through the scalar cache into SGPRs.
// Products with the sparse A = I + S and B read only rows 0..11 of T = H B and rows 0..8 of
// M = H A, broadcast through LDS (7.6 KB per element).
// Quu^-1 [Qux | Qu] is formed by Gauss-Jordan elimination without pivoting on the 24 x 49 block
// matrix whose columns live one per row lane (rows split across the halves): 24 dependent steps
// per knot (vs 72 for Cholesky + two triangular solves), each broadcasting one pivot column.
// This is the reference's explicit inverse formulation (Quu.inverse(), SinglePhase.cpp:351)
// computed as a solve; Quu is SPD whenever it passes the PSD test, so no pivoting is needed.
// PSD test: every elimination pivot (= the LDL^T pivot of Quu) must exceed 1e-9; pivots of Quu
// dominate those of the reference's Quu - 1e-9 I by 1e-9, so every Quu the reference's LDLT
// accepts passes here too.
//
// k_lin_rollout: the linear rollout that follows a successful sweep, one wave per element.
//
// Both kernels are templates on the arithmetic type `real`: double is the reference's arithmetic
// (T = double throughout HSDDPSolver); float is the fp32 Riccati mode (SURVEY.md §8 config C5:
// fp32 LQ records, fp32 sweep and linear rollout, fp64 line search / costs / outer loop).  The
// float instantiation keeps the lane mapping and uses the f32 forms of the same instructions
// (v_mov_b32_dpp / v_fmac_f32_dpp, one permlane32 swap, v_mfma_f32_16x16x4_f32).
#include <utility>

#include "hsddp_device.h"

namespace hsddp {

using namespace hkd;

constexpr int HC = 12;      // columns per half-wave; coupled controls per knot
constexpr int XS = 25;      // padded row stride of the LDS matrix (row-per-lane writes without conflicts)
constexpr int OFF_M9 = 0;  // M rows 0..8 [9][XS] in Bm until the Z rows take their place
// S.A regions (doubles): the knot's LQ record [0, LQW) until Qux_c [12][XS] takes its place;
// above it T_c = H B_c [24][12], then Quu_cc^-1 by columns [12][16], then Kp [12][XS] (each read
// before the next overwrites it).
constexpr int OFF_QX = 0;
constexpr int OFF_TC = HC * XS;
constexpr int OFF_QI = HC * XS;
constexpr int OFF_KP = HC * XS;
static_assert(LQW <= OFF_TC && OFF_TC + NX * HC <= NX * XS, "S.A layout");

#ifndef HSDDP_STAMPS
#define HSDDP_STAMPS 0
#endif

template <typename real>
struct BwdElem {
#if HSDDP_STAMPS
    unsigned long long st[10], tprev;  // diagnostic build: cycles per knot stage (lane 0)
#endif
    alignas(16) real A[NX * XS];  // LQ record copy -> Qux_c [12][XS] | Quu_cc^-1 [12][16] -> Kp [12][XS]
    real Bm[NX * XS];             // T_c = H B_c [24][12] | M rows 0..8 [9][24] -> Z rows -> symmetric Qxx -> H (stride XS)
    alignas(16) real d[NX];       // Defect[k+1] -> Qu_c
    real Gn[NX], wqu[HC];
    double red[4];
};

// Per-precision buffers: LQ record (stride LQS), compact gains and the Defect copy the sweep reads.
template <typename real> struct Prec;
template <> struct Prec<double> {
    static constexpr int LQS = LQW;
    static DEV const double *lq(const Bufs &d) { return d.lq; }
    static DEV double *K(const Bufs &d) { return d.K; }
    static DEV const double *def(const Bufs &d) { return d.Defect; }
};
template <> struct Prec<float> {
    static constexpr int LQS = LQW32;
    static DEV const float *lq(const Bufs &d) { return d.lq32; }
    static DEV float *K(const Bufs &d) { return d.K32; }
    static DEV const float *def(const Bufs &d) { return d.def32; }
};

// In-kernel stamps (diagnostic build only, -DHSDDP_STAMPS=1): s_memtime at the stage boundaries
// of a knot, the differences summed per stage by lane 0 into LDS and written to Bufs::dbg.
#if HSDDP_STAMPS
#define STAMP(n)                                                                              \
    do {                                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                                    \
        unsigned long long t_;                                                                \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");            \
        __builtin_amdgcn_sched_barrier(0);                                                    \
        if (threadIdx.x == 0) {                                                               \
            if ((n) > 0) S.st[n] += t_ - S.tprev;                                             \
            S.tprev = t_;                                                                     \
        }                                                                                     \
    } while (0)
#else
#define STAMP(n) \
    do {         \
    } while (0)
#endif

// A 64-thread workgroup is one wave, so __syncthreads() lowers to no instruction and stops no
// code motion; the memory clobber keeps each phase's LDS loads in their phase.
#define HSYNC()                        \
    do {                               \
        __syncthreads();               \
        asm volatile("" ::: "memory"); \
    } while (0)

// The same inside divergent code and where no fence may drain memory operations in flight: LDS
// operations of one wave complete in order, so a compiler barrier suffices in a one-wave group.
#define LSYNC() asm volatile("" ::: "memory")

// Compile-time loop: the body sees its index as a constant, so per-lane register arrays indexed
// by it stay in VGPRs (a runtime index would demote them to scratch).
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

// read-only, wave-uniform data: the constant address space lets the compiler use scalar loads
template <typename real>
DEV const __attribute__((address_space(4))) real *uniform_ptr(const real *p)
{
    return (const __attribute__((address_space(4))) real *)p;
}

// a value known to be equal on all lanes, moved to SGPRs
DEV double uniform(double v)
{
    const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
    const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
    return __hiloint2double(hi, lo);
}
DEV float uniform(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }

// v on lane `src` (a constant), broadcast to every lane through SGPRs
DEV double lane_value(double v, int src)
{
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
    return __hiloint2double(hi, lo);
}
DEV float lane_value(float v, int src) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src)); }

// 1 / x from the hardware reciprocal refined by two Newton steps (within an ulp of the IEEE
// quotient; 5 VALU operations instead of the ~10 of a correctly rounded division)
DEV double recip(double x)
{
    double r = __builtin_amdgcn_rcp(x);
    double e = __builtin_fma(-x, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-x, r, 1.0);
    return __builtin_fma(r, e, r);
}
// f32: v_rcp_f32 is good to 1 ulp; one Newton step
DEV float recip(float x)
{
    float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(r, e, r);
}

// value held by the same lane of the other half-wave (call with all 64 lanes active)
DEV double other_half(double v)
{
    const unsigned lo = __double2loint(v), hi = __double2hiint(v);
    const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    return threadIdx.x < 32 ? __hiloint2double(b[1], a[1]) : __hiloint2double(b[0], a[0]);
}
DEV float other_half(float v)
{
    const unsigned u = __float_as_uint(v);
    const auto a = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    return __uint_as_float(threadIdx.x < 32 ? a[1] : a[0]);
}

// v on lane j of this lane's 16-lane row (DPP row_newbcast; the s_nop gives a VGPR written by
// the previous VALU instruction its two wait states before the DPP read)
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

// w += (w on lane j of this lane's 16-lane row) * s, the broadcast fused into the FMA;
// `fresh`: w may have been written by the instruction just before
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

// D = A B + C on a 16 x 16 x 4 MFMA tile (one operand value per lane: A[l & 15][l >> 4],
// B[l >> 4][l & 15]); result register g of lane l is row mfma_row(l >> 4, g), column l & 15 —
// the f64 form interleaves rows, the f32 form blocks them (cdna_hip_programming.md, fragment layout)
typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
DEV d4 mfma16(double a, double b, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }
DEV f4 mfma16(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
template <typename real> using acc4 = std::conditional_t<sizeof(real) == 8, d4, f4>;
template <typename real>
DEV constexpr int mfma_row(int lk, int g) { return sizeof(real) == 8 ? lk + 4 * g : 4 * lk + g; }

// per-phase constants of one element
template <typename real>
struct PhaseConst {
    int c[4];
    int cmask;   // bit l = c_l: a lane-dependent leg index becomes one shift, not a select chain
    real bv[4];  // dt c_l / m     (B rows 9..11)
    real bq[4];  // dt (1 - c_l)   (B rows 12..23)
};

// Wave-uniform: contacts through the scalar cache, and selects instead of arithmetic so the
// constants stay in SGPRs (dt * c / m is dt / m or 0 exactly for c in {0, 1}).
template <typename real>
DEV void load_phase(const Params &p, const Bufs &d, size_t b, int i, PhaseConst<real> &pc)
{
    typedef const __attribute__((address_space(4))) int cint;
    cint *cs = (cint *)(d.contacts + (b * (p.P + 1) + i) * 4);
    pc.cmask = 0;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        pc.c[l] = cs[l];
        pc.cmask |= (pc.c[l] != 0) << l;
        pc.bv[l] = pc.c[l] ? (real)p.dt_m : (real)0;
        pc.bq[l] = pc.c[l] ? (real)0 : (real)p.dt;
    }
}

// lxx (dt Q + dt D^T Qfoot D, HKDCost.cpp:32) row r as: diagonal + cross terms with the foot columns
template <typename real>
struct LxxRow {
    real diag, xq[4], xp;  // xq[l]: (r in pos) x (col 12+3l+(r-3)); xp: (r in q) x (col 3+(r-12)%3)
};

// contact of leg l (runtime, lane-dependent) as 0 / 1
template <typename real>
DEV int contact(const PhaseConst<real> &pc, int l) { return (pc.cmask >> l) & 1; }

// a[i] for a runtime i, as selects (a runtime index would put the array in scratch)
template <typename T>
DEV T pick4(const T (&a)[4], int i)
{
    return i == 0 ? a[0] : i == 1 ? a[1] : i == 2 ? a[2] : a[3];
}

// a[i] for a runtime i < N, as selects over the (wave-uniform) entries
template <int N>
DEV double pick(const double (&a)[N], int i)
{
    double e[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        e[k] = a[k];
        asm volatile("" : "+s"(e[k]));  // opaque: keeps the selects from folding back into an indexed load
    }
    double v = e[0];
#pragma unroll
    for (int k = 1; k < N; ++k) v = i == k ? e[k] : v;
    return v;
}

// q_diag / foot_weight (hsddp_device.h) with the lane-dependent indices resolved by selects:
// a lane-indexed read of a kernel-argument array is a memory round trip
template <typename real>
DEV void lxx_row(const Params &p, const PhaseConst<real> &pc, int r, LxxRow<real> &L)
{
    L.diag = 0.0; L.xp = 0.0;
#pragma unroll
    for (int l = 0; l < 4; ++l) L.xq[l] = 0.0;
    if (r >= NX) return;
    double dg = p.dt * (r < 12 ? pick(p.qbase, r) : p.q_qJ * (1 - contact(pc, (r - 12) / 3)));
    if (r >= 3 && r < 6) {
        // dt c^2 (foot_gain w c) = dt foot_gain w for c = 1, else 0 (selects: no per-phase
        // conversions kept live across the knot loop)
        const double fw = p.dt * (p.foot_gain * pick(p.foot_w, r - 3));
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const double w = pc.c[l] ? fw : 0.0;
            dg += w;
            L.xq[l] = -w;
        }
    } else if (r >= 12) {
        const int m = r - 12;
        const double w = contact(pc, m / 3) ? p.dt * (p.foot_gain * pick(p.foot_w, m % 3)) : 0.0;
        dg += w;
        L.xp = -w;
    }
    L.diag = dg;
}

// lxx row r from the per-phase diagonal table (column XS - 1 of the S.Bm rows, written by
// bwd_sweep at the phase start): the foot cross terms are the negated diagonal entries of the
// stance feet's rows, -lxx[12 + 3 l + a][12 + 3 l + a] (= -dt foot_gain w_a), so no parameter
// is needed inside the knot loop
template <typename real>
DEV void lxx_row_table(const real *Bm, const PhaseConst<real> &pc, int r, LxxRow<real> &L)
{
    const int rr = r < NX ? r : 0;
    const bool pos = r >= 3 && r < 6;
    const int a = pos ? r - 3 : 0;
    // every read unconditional (then opaque): the selects below must not become branches
    real dr = Bm[rr * XS + NX], dq[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) dq[l] = Bm[(12 + 3 * l + a) * XS + NX];
    asm volatile("" : "+v"(dr), "+v"(dq[0]), "+v"(dq[1]), "+v"(dq[2]), "+v"(dq[3]));
    L.diag = r < NX ? dr : (real)0;
#pragma unroll
    for (int l = 0; l < 4; ++l) L.xq[l] = (pos && pc.c[l]) ? -dq[l] : (real)0;
    L.xp = (r >= 12 && r < NX && contact(pc, (rr - 12) / 3)) ? -dr : (real)0;
}

// lxx(r, 12 hf + i) for a compile-time i
template <int i, typename real>
DEV real lxx_half(const LxxRow<real> &L, int r, int hf)
{
    const real dg = (HC * hf + i == r) ? L.diag : (real)0;
    const real x1 = (r == 3 + i % 3) ? L.xq[i / 3] : (real)0;  // hf = 1
    real x0 = 0;                                               // hf = 0
    if constexpr (i >= 3 && i < 6) x0 = (r >= 12 && r < NX && (r - 12) % 3 == i - 3) ? L.xp : (real)0;
    return dg + (hf ? x1 : x0);
}

// out[i] = sum_j S[j][12 hf + i] col[j] for this half's 12 columns of S (= A - I; rows 0..2:
// eul, cols {1,2,6,7,8}; rows 3..5: dt at cols 9..11; rows 6..8: omega, cols {0..8, 12, 13, 15,
// 16, 18, 19, 21, 22}), S values wave-uniform from the LQ record (scalar loads)
template <typename real>
DEV void st_apply(const __attribute__((address_space(4))) real *lqs, real dt, int hf, const real (&col)[9], real (&out)[12])
{
    if (hf == 0) {
        static_for<12>([&](auto I) {
            constexpr int c = I;
            constexpr int qe = se_index(c), qw = sw_index(c);
            real v = 0;
            if constexpr (qe >= 0)
                v += lqs[LQ_SE + qe] * col[0] + lqs[LQ_SE + 5 + qe] * col[1] + lqs[LQ_SE + 10 + qe] * col[2];
            if constexpr (c >= 9) v += dt * col[c - 6];
            if constexpr (qw >= 0)
                v += lqs[LQ_SW + qw] * col[6] + lqs[LQ_SW + 17 + qw] * col[7] + lqs[LQ_SW + 34 + qw] * col[8];
            out[c] = v;
        });
    } else {
        static_for<12>([&](auto I) {
            constexpr int i = I, qw = sw_index(12 + i);
            if constexpr (qw >= 0)
                out[i] = lqs[LQ_SW + qw] * col[6] + lqs[LQ_SW + 17 + qw] * col[7] + lqs[LQ_SW + 34 + qw] * col[8];
            else
                out[i] = 0;
        });
    }
}

// Column r of S (= A - I): coefficients S[j][r], j = 0..8
template <typename real>
DEV void s_column(const real *lq, real dt, int r, real *sc)
{
    int q = (r < NX) ? se_index(r) : -1;
#pragma unroll
    for (int j = 0; j < 3; ++j) sc[j] = q >= 0 ? lq[LQ_SE + 5 * j + q] : (real)0;
#pragma unroll
    for (int j = 0; j < 3; ++j) sc[3 + j] = (r == j + 9) ? dt : (real)0;
    q = (r < NX) ? sw_index(r) : -1;
#pragma unroll
    for (int j = 0; j < 3; ++j) sc[6 + j] = q >= 0 ? lq[LQ_SW + 17 * j + q] : (real)0;
}

// one knot's LQ record (LQW doubles) and a 24-vector from global memory into LDS: every load is
// issued before the first store, so the wave waits for one memory round trip, not four
template <typename real>
DEV void stage_knot_inputs(real *lq_lds, const real *lq_g, real *v_lds, const real *v_g, int lane)
{
    static_assert(LQW > 128 && LQW <= 192, "three loads per lane");
    const real a0 = lq_g[lane], a1 = lq_g[64 + lane];
    const real a2 = lane < LQW - 128 ? lq_g[128 + lane] : (real)0;
    const real v = lane < NX ? v_g[lane] : (real)0;
    lq_lds[lane] = a0;
    lq_lds[64 + lane] = a1;
    if (lane < LQW - 128) lq_lds[128 + lane] = a2;
    if (lane < NX) v_lds[lane] = v;
}

// One knot's LQ record into S.A[0, LQW) and its Defect[k+1] into S.d by LDS-DMA (16 bytes per
// lane per instruction, contiguous from M0).  Inline asm: the compiler neither waits for it nor
// knows it writes LDS; the consumer waits with vmcnt(0) (bwd_knot).  The leading lgkmcnt(0)
// retires every LDS read of the old contents first.  (M0 is compiler-reserved: saved, set with one
// wait state before the DMA, restored.)
template <typename real>
DEV void knot_fetch(BwdElem<real> &S, const real *lq_g, const real *def_g, int lane)
{
    constexpr int E = 16 / sizeof(real);  // values per 16-byte piece
    constexpr int LP = LQW / E + (LQW % E != 0), NL = (LP + 63) / 64;  // record pieces, instructions
    static_assert(LP * E <= Prec<real>::LQS && NL <= 2 && NX % E == 0, "16-byte pieces, at most two instructions");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int t = 0; t < NL + 1; ++t) {
        const int n = t < NL ? min(64, LP - 64 * t) : NX / E;  // pieces
        if (lane < n) {
            const real *src = t < NL ? lq_g + 64 * E * t + E * lane : def_g + E * lane;
            const unsigned m0 = (unsigned)(size_t)(t < NL ? S.A + 64 * E * t : S.d);
            unsigned keep;
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep)
                         : "v"(src), "s"(m0)
                         : "memory");
        }
    }
}

template <typename real>
DEV real half_sum(real v)
{
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// One knot of SinglePhase::backward_sweep (SinglePhase.cpp:298-362).  H[k+1] rows are in S.Bm
// (stride XS) and g holds G[k+1][r] on entry; H[k] and G[k] on exit.  `live` turns false when
// Quu fails the PSD test (wave-uniform).
//
// Coupled controls: for leg l the three GRF columns of B carry a factor c_l and the three
// joint-velocity columns a factor (1 - c_l) (HKDDynamics: contact_moment, B rows 9..23), so
// exactly 12 columns of B are nonzero — control q (0..11) is u = q for a stance leg and
// u = 12 + q for a swing leg.  The other 12 controls z have B[:, z] = 0 exactly, hence
// Qux[z, :] = 0, Quu[z, :] = Quu[:, z] = 0 off the diagonal and Quu[z][z] = dt R_z + reg
// (the ReB Hessian only touches stance GRFs).  Quu is block diagonal under this permutation,
// so Quu^-1 [Qux | Qu] = [Quu_cc^-1 [Qux_c | Qu_c] ; 0 | Qu_z / Quu_zz] exactly, and the
// reference's 24-control solve reduces to a 12 x 12 one plus 12 divisions.
template <typename real>
DEV void bwd_knot(const Params &p, const Bufs &d, BwdElem<real> &S, const PhaseConst<real> &pc, size_t b, int s, int kc,
                  real *Kout, double *dUout, real reg, bool pre, bool more, bool &live, real &g, real &dV1, real &dV2)
{
    // opaque per knot: keeps LICM from hoisting lane-dependent constants of the knot body
    // (regularised diagonals, lxx entries) out of the knot loop into long-lived VGPRs
    int lane = threadIdx.x;
    asm volatile("" : "+v"(lane));
    asm volatile("" : "+v"(reg));
    const int r = lane & 31, hf = lane >> 5, cb = HC * hf;
    const bool rowl = r < NX;
    const int pos = lane & 15, R = lane >> 4;  // position in the 16-lane DPP row R
    const bool qr = pos < HC;                    // elimination column pos of Quu_cc (all four rows)
    const bool il = pos >= HC && R < 3;          // elimination column ic of the identity
    const int ic = il ? 4 * R + pos - HC : 0;
    const bool ul = lane == 60;                  // elimination column Qu_c
    const bool ql = hf == 1 && r < HC;           // decoupled control z(r)
    const real dt = p.dt;
    const size_t kq = b * p.Kc + kc;
    STAMP(0);
    constexpr int LQS = Prec<real>::LQS;
    const real *lqg = Prec<real>::lq(d), *defg = Prec<real>::def(d);
    const auto lqs = uniform_ptr(lqg + kq * LQS);
    real *lq = S.A;  // LDS copy for lane-indexed reads
    if (pre) // the previous knot requested this one's LQ record and Defect (knot_fetch)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else
        stage_knot_inputs(lq, lqg + kq * LQS, S.d, defg + (b * p.S + s + 1) * NX, lane);
    real h[HC];  // this lane's columns of H[k+1] row r
#pragma unroll
    for (int i = 0; i < HC; ++i) h[i] = rowl ? S.Bm[r * XS + cb + i] : (real)0;
    HSYNC();
    STAMP(1);
    // Gnext = G + H Defect[k+1] (SinglePhase.cpp:320)
    real part = 0.0;
#pragma unroll
    for (int i = 0; i < HC; ++i) part += h[i] * S.d[cb + i];
    const real gn = g + (part + other_half(part));
    // M = H A on this half's columns (the second half needs H[r][6..8] from the first);
    // T_c = H B_c, each coupled column written by the half that holds its H entries
    real h68[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) h68[j] = other_half(h[6 + j]);
    // (for a swing leg the first half's GRF column value is exactly 0, for a stance leg the second
    // half's joint-velocity value is: each half stores only the columns it owns)
    real m[HC], tc[HC];
    if (hf == 0) {
        static_for<HC>([&](auto I) {
            constexpr int c = I;
            real v = h[c];
            constexpr int qe = se_index(c), qw = sw_index(c);
            if constexpr (qe >= 0)
                v += h[0] * lqs[LQ_SE + qe] + h[1] * lqs[LQ_SE + 5 + qe] + h[2] * lqs[LQ_SE + 10 + qe];
            if constexpr (c >= 9) v += h[c - 6] * dt;
            if constexpr (qw >= 0)
                v += h[6] * lqs[LQ_SW + qw] + h[7] * lqs[LQ_SW + 17 + qw] + h[8] * lqs[LQ_SW + 34 + qw];
            m[c] = v;
            tc[c] = h[6] * lqs[LQ_BW + c] + h[7] * lqs[LQ_BW + 12 + c] + h[8] * lqs[LQ_BW + 24 + c] +
                    h[9 + c % 3] * pc.bv[c / 3];
        });
    } else {
        static_for<HC>([&](auto I) {
            constexpr int i = I;
            real v = h[i];
            constexpr int qw = sw_index(HC + i);
            if constexpr (qw >= 0)
                v += h68[0] * lqs[LQ_SW + qw] + h68[1] * lqs[LQ_SW + 17 + qw] + h68[2] * lqs[LQ_SW + 34 + qw];
            m[i] = v;
            tc[i] = h[i] * pc.bq[i / 3];
        });
    }
    pin(m);
    pin(tc);
    // T_c[r][q] = the two halves' values summed (one of them is exactly 0): every lane gets the
    // full row, half 0 stores columns 0..5 and half 1 columns 6..11 (no branch on the contacts)
#pragma unroll
    for (int q = 0; q < HC; ++q) tc[q] += other_half(tc[q]);
    if (rowl)
#pragma unroll
        for (int i = 0; i < HC / 2; ++i) S.A[OFF_TC + r * HC + HC / 2 * hf + i] = hf ? tc[HC / 2 + i] : tc[i];
    if (r < 9)
#pragma unroll
        for (int i = 0; i < HC; ++i) S.Bm[OFF_M9 + r * XS + cb + i] = m[i];
    if (lane < NX) S.Gn[lane] = gn;
    HSYNC();
    SFENCE();
    STAMP(2);
    // Qx, Qxx = lxx + A^T M, and the coupled blocks Qux_c, Quu_cc, Qu_c
    // (SinglePhase.cpp:323-327; regularisation on both diagonals, MultiPhaseDDP.cpp:160).
    // The S^T X products (S = A - I) are evaluated transposed: a lane gathers one column of X
    // and applies S, whose sparsity is known at compile time and whose values are wave-uniform
    // (SGPRs) — 9 LDS reads per product instead of one broadcast read per multiply.
    real sc[9];
    s_column(lq, dt, r, sc);
    real qx = 0.0;
    if (rowl) {
        real a = 0.0;
#pragma unroll
        for (int j = 0; j < 9; ++j) a += sc[j] * S.Gn[j];
        qx = lq[LQ_LX + r] + (gn + a);
    }
    // lane-indexed coefficients of control rq (the Quu row / decoupled-control lanes): leg lr,
    // axis ar, B_c column rq (rows 6..8 from the LQ record, row 9 + ar or 12 + rq from the contact)
    const int rq = qr ? pos : 0;
    const int lr = rq / 3, ar = rq % 3;
    const bool stz = contact(pc, lr) != 0;
    real rb3[3];  // row ar of leg lr's ReB Hessian block, stored (00,01,02,11,12,22)
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const int lo = min(a, ar), hi = max(a, ar);
        rb3[a] = lq[LQ_RB + 6 * lr + (lo == 0 ? hi : lo == 1 ? 2 + hi : 5)];
    }
    const real bw0 = lq[LQ_BW + rq], bw1 = lq[LQ_BW + 12 + rq], bw2 = lq[LQ_BW + 24 + rq];
    // decoupled control z(r) on the ql lanes: Qu_z, Quu_zz
    const real qzz = dt * (real)(stz ? p.r_qJd : p.r_grf) + reg;
    const real quz = lq[LQ_LU + (stz ? HC + rq : rq)];
    // Qu_c[q] = lu_c + B_c^T Gnext on lane q < 12 (into S.d)
    if (lane < HC) {
        const real gb = stz ? (bw0 * S.Gn[6] + bw1 * S.Gn[7] + bw2 * S.Gn[8]) + (real)p.dt_m * S.Gn[9 + ar]
                              : dt * S.Gn[HC + rq];
        S.d[lane] = lq[LQ_LU + (stz ? rq : HC + rq)] + gb;
    }
    // Z = M + (S^T M9)^T on this lane's row: Qxx = lxx + Z^T-symmetric part (below)
    real z[HC];
    {
        const int rr = rowl ? r : 0;
        real col[9], y[HC];
#pragma unroll
        for (int j = 0; j < 9; ++j) col[j] = S.Bm[OFF_M9 + j * XS + rr];
        st_apply(lqs, dt, hf, col, y);
#pragma unroll
        for (int i = 0; i < HC; ++i) z[i] = m[i] + y[i];
    }
    HSYNC();  // the LQ copy and M9 are dead: S.A takes Qux_c below T_c, Bm the Z rows
    STAMP(3);
    if (rowl)
#pragma unroll
        for (int i = 0; i < HC; ++i) S.Bm[r * XS + cb + i] = z[i];
    {
        // Qux_c^T = A^T T_c = T_c + S^T T_c: lane (hf, q < 12) forms column q of S^T T_c on its
        // half's rows and writes row q of Qux_c [12][XS] (its half's columns); every read is
        // issued before the first write
        const int rt = r < HC ? r : 0;
        real col[9], y[HC], t[HC];
#pragma unroll
        for (int j = 0; j < 9; ++j) col[j] = S.A[OFF_TC + j * HC + rt];
#pragma unroll
        for (int i = 0; i < HC; ++i) t[i] = S.A[OFF_TC + (cb + i) * HC + rt];
        st_apply(lqs, dt, hf, col, y);
        if (r < HC)
#pragma unroll
            for (int i = 0; i < HC; ++i) S.A[OFF_QX + r * XS + cb + i] = t[i] + y[i];
    }
    HSYNC();
    STAMP(4);
    // Qxx = lxx + M + S^T M9 and lxx is symmetric, so (Qxx + Qxx^T) / 2 (SinglePhase.cpp:352)
    // = lxx + (Z + Z^T) / 2, symmetrised in place: every lane reads its row and its 12 transposed
    // entries before any lane writes
    if (rowl) {
        LxxRow<real> lx_;
        lxx_row_table(S.Bm, pc, r, lx_);
        real zt[HC], zo[HC];
#pragma unroll
        for (int i = 0; i < HC; ++i) {
            zt[i] = S.Bm[(cb + i) * XS + r];
            zo[i] = S.Bm[r * XS + cb + i];
        }
        LSYNC();
        static_for<HC>([&](auto I) {
            constexpr int i = I;
            const int c = cb + i;
            S.Bm[r * XS + c] = lxx_half<i>(lx_, r, hf) + (c == r ? reg : (real)0) + (zo[i] + zt[i]) / 2;
        });
    }
    STAMP(5);
    // elimination operand, one column of [Quu_cc | I | Qu_c] per lane: lane 16 R + j (j < 12)
    // holds Quu_cc = luu + B_c^T T_c + reg I as row j (B_c column j against the rows of T_c:
    // lane-indexed coefficients, broadcast rows, no scalar loads) in each of the four 16-lane DPP
    // rows R, lanes 16 R + 12 + t (R < 3) column 4 R + t of the identity, lane 60 Qu_c
    // (SinglePhase.cpp:323-327; regularisation MultiPhaseDDP.cpp:160)
    real w[HC];
    {
        const real bv = stz ? (real)p.dt_m : (real)0, bq = stz ? (real)0 : dt;
        const real ld = dt * (real)(stz ? p.r_grf : p.r_qJd);
        const real *t6 = S.A + OFF_TC + 6 * HC, *t9 = S.A + OFF_TC + (9 + ar) * HC,
                     *tq = S.A + OFF_TC + (HC + rq) * HC;
        // B_c column rq is (bw0, bw1, bw2, bv) on rows 6, 7, 8, 9 + ar for a stance leg and bq on
        // row 12 + rq for a swing leg, the other entries exactly 0 (HKDDynamics: c_l factors), so
        // the stance and swing sums add exact zeros: one select-free formula, every read
        // unconditional (a select on a loaded value becomes a branch around the load)
        const real ul1 = ul ? (real)1 : (real)0;
        static_for<HC>([&](auto I) {
            constexpr int c = I;
            const real vb = bw0 * t6[c] + bw1 * t6[HC + c] + bw2 * t6[2 * HC + c] + bv * t9[c] + bq * tq[c];
            const real lu = (c == rq ? ld : (real)0) + ((stz && c / 3 == lr) ? rb3[c % 3] : (real)0);
            const real vu = lu + vb + (c == rq ? reg : (real)0);
            const real vo = (il && c == ic ? (real)1 : (real)0) + ul1 * S.d[c];
            w[c] = qr ? vu : vo;
        });
    }
    STAMP(6);
    // PSD test (LDLT of Quu - 1e-9 I, SinglePhase.cpp:342-348): the decoupled diagonal, then
    // every Gauss-Jordan pivot of the coupled block.  ballot is convergent, so each test stays
    // in its step.
    unsigned long long bad = __builtin_amdgcn_ballot_w64(ql && !(qzz > (real)1e-9));
    // Gauss-Jordan without pivoting (Quu_cc is SPD when it passes): step j takes column j of
    // Quu_cc from position j of the lane's own DPP row (row_newbcast, fused into the FMA), so no
    // value leaves the VALU.  Afterwards the identity lanes hold Quu_cc^-1 — the reference's
    // explicit inverse (Quu.inverse(), SinglePhase.cpp:351) — and lane 60 Quu_cc^-1 Qu_c.
    static_for<HC>([&](auto J) {
        constexpr int j = J;
        const real piv = row_bcast<j>(w[j]);
        bad |= __builtin_amdgcn_ballot_w64(!(piv > (real)1e-9));
        const real f = w[j] * recip(piv), nf = -f;
        static_for<HC>([&](auto I) {
            constexpr int i = I;
            if constexpr (i != j) fmac_row_bcast<j, i == (j + HC - 1) % HC>(w[i], nf);
        });
        w[j] = f;
        SFENCE();
    });
    STAMP(7);
    live = live && bad == 0;
    if (!live) return;
    // Quu_cc^-1 by columns [c][16] (rows 12..15 read as zero) and Quu_cc^-1 Qu_c into LDS
    if (il)
#pragma unroll
        for (int q = 0; q < HC; ++q) S.A[OFF_QI + ic * 16 + q] = w[q];
    if (ul)
#pragma unroll
        for (int q = 0; q < HC; ++q) S.wqu[q] = w[q];
    // dU = -Quu^-1 Qu: coupled controls from lane 60, decoupled ones (Qu_z / Quu_zz) from the ql lanes
    double *dUg = dUout + (size_t)kc * NX;
    if (ul)
        static_for<HC>([&](auto I) {
            constexpr int q = I;
            dUg[pc.c[q / 3] ? q : HC + q] = -w[q];
        });
    real dvp = 0.0;
    if (ql) {
        const real duz = quz / qzz;
        dUg[contact(pc, r / 3) ? HC + r : r] = -duz;
        dvp = quz * duz;
    }
    HSYNC();
    const int li = lane & 15, lk = lane >> 4;
    // Kp = Quu_cc^-1 Qux_c (12 x 24, K = 12) on the matrix cores (v_mfma_f64_16x16x4_f64; operands
    // A[l & 15][k = l >> 4], B[k = l >> 4][l & 15]; result rows (l >> 4) + 4 reg, column l & 15):
    // into LDS for the value update, and K = -Kp to the compact gain rows (KCW layout)
    {
        acc4<real> k0 = {0, 0, 0, 0}, k1 = k0;
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) {
            const int c = 4 * ks + lk;
            const real a = li < HC ? S.A[OFF_QI + c * 16 + li] : (real)0;
            const real b0 = S.A[OFF_QX + c * XS + li], b1 = S.A[OFF_QX + c * XS + 16 + li];
            k0 = mfma16(a, b0, k0);
            k1 = mfma16(a, b1, k1);
        }
        HSYNC();  // Quu^-1 is read; Kp takes its place
        real *Kg = Kout + (size_t)kc * KCW;
        // rows 0..11 hold the result: registers 0..2 in the f64 layout, 0..3 (rows < 12) in the f32 one
#pragma unroll
        for (int g = 0; g < (sizeof(real) == 8 ? 3 : 4); ++g) {
            const int q = mfma_row<real>(lk, g);
            if (sizeof(real) == 4 && q >= HC) continue;
            S.A[OFF_KP + q * XS + li] = k0[g];
            Kg[q * NX + li] = -k0[g];
            if (li < NX - 16) {
                S.A[OFF_KP + q * XS + 16 + li] = k1[g];
                Kg[q * NX + 16 + li] = -k1[g];
            }
        }
    }
    HSYNC();
    STAMP(8);
    if (ul)
#pragma unroll
        for (int q = 0; q < HC; ++q) dvp += S.d[q] * S.wqu[q];
    // expected cost change Qu^T Quu^-1 Qu (SinglePhase.cpp:357-358): half 1 holds every term
    const real dvk = lane_value(half_sum(dvp), 32);
    dV1 -= dvk;
    dV2 += dvk;
    // G = Qx - Qux_c^T Quu_cc^-1 Qu_c, H = Qxx - Qux_c^T Quu_cc^-1 Qux_c (SinglePhase.cpp:359-361)
    const int rr = rowl ? r : 0;
    real gp = 0.0;
#pragma unroll
    for (int q = 0; q < HC; ++q) gp += S.A[OFF_QX + q * XS + rr] * S.wqu[q];
    g = rowl ? qx - gp : (real)0;
    // P = Qux_c^T Kp (24 x 24, K = 12) on the matrix cores over the output tiles (0,0), (0,1) and
    // (1,1) — P is symmetric, tile (1,0) is (0,1)^T — rows / columns 24..31 are padding.  H = Qxx - P
    // is formed in place of Qxx in LDS (each entry read and written by one lane), then read back
    // as rows.
    {
        acc4<real> t00 = {0, 0, 0, 0}, t01 = t00, t11 = t00;
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) {
            const int q = 4 * ks + lk;
            const real a0 = S.A[OFF_QX + q * XS + li], a1 = S.A[OFF_QX + q * XS + 16 + li];
            const real b0 = S.A[OFF_KP + q * XS + li], b1 = S.A[OFF_KP + q * XS + 16 + li];
            t00 = mfma16(a0, b0, t00);
            t01 = mfma16(a0, b1, t01);
            t11 = mfma16(a1, b1, t11);
        }
        // S.A and S.d are read: request the next knot's inputs into them (in flight during the
        // H update and the knot transition)
        if (more) knot_fetch(S, lqg + (kq - 1) * LQS, defg + (b * p.S + s) * NX, lane);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int r0 = mfma_row<real>(lk, g), r1 = 16 + r0, c1 = 16 + li;
            S.Bm[r0 * XS + li] -= t00[g];
            if (c1 < NX) {
                S.Bm[r0 * XS + c1] -= t01[g];
                S.Bm[c1 * XS + r0] -= t01[g];
            }
            if (r1 < NX && c1 < NX) S.Bm[r1 * XS + c1] -= t11[g];
        }
    }
    HSYNC();
    STAMP(9);
}

// MultiPhaseDDP::backward_sweep (MultiPhaseDDP.cpp:190-229) with one regularisation value; the
// gains and dU rows of element b go to Kout / dUout (row kc at kc * KCW / kc * 24).
// Returns -1, or (and stops at) the control slot of the first knot whose Quu fails the PSD test:
// rows above it were written, it and the rows below were not.
template <typename real>
DEV int bwd_sweep(const Params &p, const Bufs &d, BwdElem<real> &S, size_t b, real *Kout, double *dUout, real reg,
                  real &dV1, real &dV2)
{
    const int lane = threadIdx.x, r = lane & 31, hf = lane >> 5, cb = HC * hf;
    const bool rowl = r < NX;
    real g = 0.0;  // G[r]; the value Hessian H stays in S.Bm rows
    bool live = true;
    dV1 = 0.0; dV2 = 0.0;
    for (int i = p.P - 1; i >= 0; --i) {
        PhaseConst<real> pc;
        load_phase(p, d, b, i, pc);
        const double *rec = d.term + (b * p.P + i) * TW;
        real h[HC];
        if (i == p.P - 1) {
#pragma unroll
            for (int c = 0; c < HC; ++c) h[c] = rowl ? (real)rec[TM_PHIXX + r * NX + cb + c] : (real)0;
            g = rowl ? (real)rec[TM_PHIX + r] : (real)0;
        } else {
            // impact-aware step G' = Phix + Px^T G0, H' = Phixx + Px^T H0 Px
            // (MultiPhaseDDP.cpp:480-484): W = H0 Px into S.A, then Px^T W.
            const double *Px = rec + TM_PX;
            if (lane < NX) S.Gn[lane] = g;
            real w[HC];
#pragma unroll
            for (int c = 0; c < HC; ++c) w[c] = 0.0;
            if (rowl)
                for (int k = 0; k < NX; ++k) {
                    const real hk = S.Bm[r * XS + k];
#pragma unroll
                    for (int c = 0; c < HC; ++c) w[c] += hk * (real)Px[k * NX + cb + c];
                }
            if (rowl)
#pragma unroll
                for (int c = 0; c < HC; ++c) S.A[r * XS + cb + c] = w[c];
            HSYNC();
            real gp = 0.0;
#pragma unroll
            for (int c = 0; c < HC; ++c) w[c] = 0.0;
            if (rowl)
                for (int j = 0; j < NX; ++j) {
                    const real pj = (real)Px[j * NX + r];
                    gp += pj * S.Gn[j];
#pragma unroll
                    for (int c = 0; c < HC; ++c) w[c] += pj * S.A[j * XS + cb + c];
                }
#pragma unroll
            for (int c = 0; c < HC; ++c) h[c] = rowl ? (real)rec[TM_PHIXX + r * NX + cb + c] + w[c] : (real)0;
            g = rowl ? (real)rec[TM_PHIX + r] + gp : (real)0;
        }
        HSYNC();
        if (rowl)
#pragma unroll
            for (int c = 0; c < HC; ++c) S.Bm[r * XS + cb + c] = h[c];
        if (rowl && hf == 0) { // this phase's lxx diagonal into the padding column (lxx_row_table)
            LxxRow<real> lx_;
            lxx_row(p, pc, r, lx_);
            S.Bm[r * XS + NX] = lx_.diag;
        }
        HSYNC();
        const int N = p.N[i], s0 = p.s0[i], k0 = p.k0[i];
        int k = N - 1;
#pragma unroll 1
        for (; k >= 0; --k) {
            bwd_knot(p, d, S, pc, b, s0 + k, k0 + k, Kout, dUout, reg, k < N - 1, k > 0, live, g, dV1, dV2);
            if (!live) break;
        }
        if (!live) return k0 + k;
        // G[0] += H[0] Defect[0] (SinglePhase.cpp:365)
        if (lane < NX) S.d[lane] = Prec<real>::def(d)[(b * p.S + s0) * NX + lane];
        HSYNC();
        real a = 0.0;
        if (rowl)
#pragma unroll
            for (int c = 0; c < HC; ++c) a += S.Bm[r * XS + cb + c] * S.d[cb + c];
        a += other_half(a);
        if (rowl) g += a;
        HSYNC();
    }
    return -1;
}

template <typename real>
__global__ __launch_bounds__(64, 4) void k_riccati(Params p, Bufs d)
{
    __shared__ BwdElem<real> S;
    const int lane = threadIdx.x;
    const size_t b = blockIdx.x;
    ElemState &E = d.el[b];
    if (E.done || E.inner_done) return;
#if HSDDP_STAMPS
    if (lane < 10) S.st[lane] = 0;
#endif
    // compute_cost + feasibility at the start of the inner iteration (MultiPhaseDDP.cpp:306-307)
    if (lane == 0) {
        double cost = 0.0, feas = 0.0;
        for (int i = 0; i < p.P; ++i) {
            double ci = 0.0, fi = 0.0;
            for (int k = 0; k < p.N[i]; ++k) ci += d.slot_cost[b * p.S + p.s0[i] + k];
            ci += d.slot_cost[b * p.S + p.s0[i] + p.N[i]];
            for (int k = 0; k <= p.N[i]; ++k) fi += d.slot_feas[b * p.S + p.s0[i] + k];
            cost += ci;
            feas += fi;
        }
        S.red[0] = cost;
        S.red[1] = sqrt(feas);
    }
    HSYNC();
    const double cost = uniform(S.red[0]), feas = uniform(S.red[1]);
    double reg = uniform(E.reg);
    real dV1 = 0, dV2 = 0;
    real *Ko = Prec<real>::K(d) + b * p.Kc * KCW;
    double *dUo = d.dU + b * p.Kc * NX;
    // backward_sweep_regularized (MultiPhaseDDP.cpp:141-181): the sweep with the element's mu,
    // then mu = max(mu * update_regularization, 1e-3) until a sweep succeeds or mu > 1e2
    bool ok = false;
    for (bool first = true;; first = false) {  // one call site: the sweep is inlined once
        if (bwd_sweep(p, d, S, b, Ko, dUo, (real)reg, dV1, dV2) < 0) { ok = true; break; }
        if (first && p.retry_cap > 0) {
            // the retries run in parallel in k_riccati_retry (the first retry_cap failures of
            // this launch); k_riccati_select then takes the first mu that succeeds, as the loop
            // would
            if (lane == 0) {
                const int f = atomicAdd(d.retry_count, 1);
                if (f < p.retry_cap) d.retry_list[f] = RetryEntry{(int)b, 0, reg};
                S.red[2] = f;
            }
            HSYNC();
            if ((int)uniform(S.red[2]) < p.retry_cap) {
                if (lane == 0) { E.iters += 1; E.cost = cost; E.feas = feas; E.accepted = 0; }
                return;
            }
        }
        reg = fmax(reg * p.update_regularization, 1e-03);
        if (reg > 1e2) break;
    }
    reg = reg / 20;
    if (reg < 1e-06) reg = 0;
#if HSDDP_STAMPS
    HSYNC();
    if (lane < 10) d.dbg[b * 16 + lane] += S.st[lane];
#endif
    if (lane == 0) {
        E.iters += 1; E.cost = cost; E.feas = feas; E.reg = reg; E.accepted = 0;
        if (!ok) { E.status = 1; E.done = 1; E.ls_active = 0; } // goto bad_solve
    }
}

// The retries of backward_sweep_regularized for the elements k_riccati deferred, all at once:
// block (f, a) sweeps deferred element f with the a-th next mu of the schedule (a = 1 ..
// retry_m) into its own scratch rows.  Every attempt is the same deterministic sweep the
// sequential loop would run with that mu, so taking the first success (k_riccati_select) gives
// the loop's result; a straggler needing many retries costs one sweep instead of many.
template <typename real>
__global__ __launch_bounds__(64, 4) void k_riccati_retry(Params p, Bufs d)
{
    __shared__ BwdElem<real> S;
    const int f = blockIdx.x / p.retry_m, a = blockIdx.x % p.retry_m + 1;
    if (f >= min(*d.retry_count, p.retry_cap)) return;
    const RetryEntry e = d.retry_list[f];
    double reg = e.reg;
    for (int t = 0; t < a; ++t) reg = fmax(reg * p.update_regularization, 1e-03);
    int *flag = d.retry_flag + f * p.retry_m + (a - 1);
    if (reg > 1e2) {  // past the loop's exit: never tried (the schedule is non-decreasing)
        if (threadIdx.x == 0) *flag = 2;
        return;
    }
    const size_t slot = (size_t)f * p.retry_m + (a - 1);
    real dV1, dV2;
    const int fk = bwd_sweep(p, d, S, e.b, (real *)d.retry_K + slot * p.Kc * KCW, d.retry_dU + slot * p.Kc * NX,
                             (real)reg, dV1, dV2);
    if (threadIdx.x == 0) *flag = fk < 0 ? 1 : -1 - fk;  // success, or -1 - (the failing control slot)
}

// The outcome of backward_sweep_regularized for each deferred element: the first attempt that
// succeeded (its gains and dU rows copied to the element), mu / 20 (0 below 1e-6) as the next
// regularisation; when none succeeds (mu passed 1e2: status 1, bad_solve) the element's rows are
// left as the sequential loop leaves them: row kc from the last attempt that got past it.
template <typename real>
__global__ __launch_bounds__(64) void k_riccati_select(Params p, Bufs d)
{
    const int f = blockIdx.x, lane = threadIdx.x;
    if (f >= min(*d.retry_count, p.retry_cap)) return;
    const RetryEntry e = d.retry_list[f];
    const size_t b = e.b;
    double reg = e.reg;
    int win = 0;
    for (int a = 1; a <= p.retry_m; ++a) {
        reg = fmax(reg * p.update_regularization, 1e-03);
        if (reg > 1e2) break;
        if (d.retry_flag[f * p.retry_m + a - 1] == 1) { win = a; break; }
    }
    real *Ko = Prec<real>::K(d) + b * p.Kc * KCW;
    double *dUo = d.dU + b * p.Kc * NX;
    if (win) {
        const size_t slot = (size_t)f * p.retry_m + (win - 1);
        const real *Ks = (const real *)d.retry_K + slot * p.Kc * KCW;
        const double *Us = d.retry_dU + slot * p.Kc * NX;
        for (size_t q = lane; q < (size_t)p.Kc * KCW; q += 64) Ko[q] = Ks[q];
        for (size_t q = lane; q < (size_t)p.Kc * NX; q += 64) dUo[q] = Us[q];
    } else {
        const int *fl = d.retry_flag + f * p.retry_m;
        // attempt a wrote the rows above its failing slot -1 - fl[a - 1]; attempts stop at flag 2
        auto source = [&](int kc) {
            int src = 0;
            for (int a = 1; a <= p.retry_m && fl[a - 1] != 2; ++a)
                if (-1 - fl[a - 1] < kc) src = a;
            return src;
        };
        const real *K0 = (const real *)d.retry_K + (size_t)f * p.retry_m * p.Kc * KCW;
        const double *U0 = d.retry_dU + (size_t)f * p.retry_m * p.Kc * NX;
        for (size_t q = lane; q < (size_t)p.Kc * KCW; q += 64) {
            const int a = source((int)(q / KCW));
            if (a) Ko[q] = K0[(size_t)(a - 1) * p.Kc * KCW + q];
        }
        for (size_t q = lane; q < (size_t)p.Kc * NX; q += 64) {
            const int a = source((int)(q / NX));
            if (a) dUo[q] = U0[(size_t)(a - 1) * p.Kc * NX + q];
        }
    }
    if (lane == 0) {
        ElemState &E = d.el[b];
        double rn = reg / 20;
        if (rn < 1e-06) rn = 0;
        E.reg = rn;
        if (!win) { E.status = 1; E.done = 1; E.ls_active = 0; }  // goto bad_solve
    }
}

// ---------------------------------------------------------------------------------------------
// MultiPhaseDDP::linear_rollout(1.0): dX, du = dU + K dX, and the expected cost change (quirk
// A3: it replaces the sweep's dV), then the merit function (MultiPhaseDDP.cpp:309-318).
// Lanes r < 24 of each half compute row r of the same vectors; the first half stores them.
// A knot's inputs (compact K, LQ record, Defect[k+1], dU) are one LDS image (4080 bytes in fp64,
// 2144 in the fp32 mode) filled by 16-byte-per-lane LDS-DMA loads (global_load_lds_dwordx4, four
// or three instructions); the next knot's image is loaded into the other buffer while this knot
// computes.
template <typename real>
struct LinImg {
    static constexpr int K = 0;                                       // byte offsets
    static constexpr int LQ = K + KCW * (int)sizeof(real);
    static constexpr int D = LQ + Prec<real>::LQS * (int)sizeof(real);
    static constexpr int DU = D + NX * (int)sizeof(real);
    static constexpr int END = DU + NX * 8;                           // dU stays fp64
    static constexpr int NI = (END / 16 + 63) / 64;                   // DMA instructions
    static_assert(LQ % 16 == 0 && D % 16 == 0 && DU % 16 == 0 && END % 16 == 0 && NI <= 4, "16-byte pieces");
};
template <typename real>
struct LinBuf {
    alignas(16) char v[LinImg<real>::NI * 64 * 16];
};
template <typename real>
struct LinElem {
    real dx[NX], du[NX];
};

// Issued as inline asm so the waitcnt pass does not track the LDS writes (it would otherwise wait
// for every DMA in flight before any LDS read); lin_knot waits explicitly.  LDS destination of
// piece t: M0 + 16 * lane, contiguous.
template <typename real>
DEV void lin_fetch(LinBuf<real> &buf, const Params &p, const Bufs &d, size_t b, int s, int kc, int lane)
{
    using I = LinImg<real>;
    const size_t kq = b * p.Kc + kc;
    // one base per segment, biased so that base + o addresses image byte o
    const size_t kB = (size_t)(Prec<real>::K(d) + kq * KCW) - I::K,
                 lB = (size_t)(Prec<real>::lq(d) + kq * Prec<real>::LQS) - I::LQ,
                 dB = (size_t)(Prec<real>::def(d) + (b * p.S + s + 1) * NX) - I::D,
                 uB = (size_t)(d.dU + kq * NX) - I::DU;
#pragma unroll
    for (int t = 0; t < I::NI; ++t) {
        int o = 16 * (64 * t + lane);    // first byte of this lane's 16-byte piece
        o = o < I::END ? o : I::END - 16;  // spare pieces repeat the last
        const size_t base = o < I::LQ ? kB : o < I::D ? lB : o < I::DU ? dB : uB;
        const char *src = (const char *)(base + (size_t)o);
        const unsigned m0 = (unsigned)(size_t)(buf.v + 1024 * t);
        unsigned keep;  // M0 is compiler-reserved: saved, set (one wait state before the DMA), restored
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(src), "s"(m0)
                     : "memory");
    }
}

// one knot of SinglePhase::linear_rollout (SinglePhase.cpp:144-178) from the LDS image `cur`;
// when `more`, the next knot's image is requested into `nxt` first
template <typename real>
DEV void lin_knot(const Params &p, const Bufs &d, LinElem<real> &S, LinBuf<real> &cur, LinBuf<real> &nxt, bool more,
                  size_t b, int s, int kc, const PhaseConst<real> &pc, const LxxRow<real> &lx_, real ru, bool cpl,
                  int krow0, real &dx, real &v1, real &v2)
{
    using I = LinImg<real>;
    const int lane = threadIdx.x, r = lane & 31, hf = lane >> 5, cb = HC * hf;
    const bool rowl = r < NX, st = rowl && hf == 0;
    const int rr = rowl ? r : 0;
    const real dt = p.dt;
    if (more) {
        lin_fetch(nxt, p, d, b, s + 1, kc + 1, lane);
        // all but the I::NI just issued
        if constexpr (I::NI == 4)
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    static_assert(I::NI == 4 || I::NI == 3, "waitcnt above");
    LSYNC();
    const real *kimg = (const real *)(cur.v + I::K), *lq = (const real *)(cur.v + I::LQ),
               *dd = (const real *)(cur.v + I::D);
    const double *dUi = (const double *)(cur.v + I::DU);
    real krow[HC];
#pragma unroll
    for (int c = 0; c < HC; ++c) krow[c] = cpl ? kimg[krow0 + c] : (real)0;
    const real dUr = (real)dUi[rr];
    if (lane < NX) S.dx[lane] = dx;
    LSYNC();
    real kd = 0;
#pragma unroll
    for (int c = 0; c < HC; ++c) kd += krow[c] * S.dx[cb + c];
    kd += other_half(kd);
    const real du = dUr + kd;
    if (lane < NX) S.du[lane] = du;
    LSYNC();
    real nx = 0, q1 = 0, q2 = 0;
    if (rowl) {
        real sdx = 0;
        if (r < 3) {
#pragma unroll
            for (int q = 0; q < 5; ++q) sdx += lq[LQ_SE + 5 * r + q] * S.dx[se_col(q)];
        } else if (r < 6) {
            sdx = dt * S.dx[r + 6];
        } else if (r < 9) {
#pragma unroll
            for (int q = 0; q < 17; ++q) sdx += lq[LQ_SW + 17 * (r - 6) + q] * S.dx[sw_col(q)];
        }
        real bdu = 0, lxd = lx_.diag * dx, lud = ru * du;
        if (r < 6) {
            if (r >= 3) {
#pragma unroll
                for (int l = 0; l < 4; ++l) lxd += lx_.xq[l] * S.dx[12 + 3 * l + r - 3];
            }
        } else if (r < 9) {
#pragma unroll
            for (int c = 0; c < 12; ++c) bdu += lq[LQ_BW + 12 * (r - 6) + c] * S.du[c];
        } else if (r < 12) {
#pragma unroll
            for (int l = 0; l < 4; ++l) bdu += pc.bv[l] * S.du[3 * l + r - 9];
        } else {
            bdu = pick4(pc.bq, (r - 12) / 3) * S.du[r];
            lxd += lx_.xp * S.dx[3 + (r - 12) % 3];
        }
        if (r < 12) {
            const real *rb = lq + LQ_RB + 6 * (r / 3);
            const int a = r % 3, u0 = 3 * (r / 3);
            const real b0 = a == 0 ? rb[0] : a == 1 ? rb[1] : rb[2];
            const real b1 = a == 0 ? rb[1] : a == 1 ? rb[3] : rb[4];
            const real b2 = a == 0 ? rb[2] : a == 1 ? rb[4] : rb[5];
            lud += b0 * S.du[u0] + b1 * S.du[u0 + 1] + b2 * S.du[u0 + 2];
        }
        nx = (dx + sdx) + bdu + dd[r];
        q1 = lq[LQ_LX + r] * dx + lq[LQ_LU + r] * du;
        q2 = dx * lxd + du * lud;
        if (st) {
            const size_t kq = b * p.Kc + kc;
            d.du[kq * NX + r] = du;
            d.dX[(b * p.S + s + 1) * NX + r] = nx;
        }
    }
    v1 += half_sum(q1);
    v2 += half_sum(q2);
    dx = nx;
    LSYNC();
}

template <typename real>
__global__ __launch_bounds__(64) void k_lin_rollout(Params p, Bufs d)
{
    __shared__ LinElem<real> S;
    __shared__ LinBuf<real> B0;
    __shared__ LinBuf<real> B1;
    const int lane = threadIdx.x, r = lane & 31, hf = lane >> 5, cb = HC * hf;
    const size_t b = blockIdx.x;
    ElemState &E = d.el[b];
    if (E.done || E.inner_done) return;
    const bool rowl = r < NX, st = rowl && hf == 0;
    const int rr = rowl ? r : 0;
    const real *defg = Prec<real>::def(d);
    real v1 = 0, v2 = 0, dx = 0;
    for (int i = 0; i < p.P; ++i) {
        PhaseConst<real> pc;
        load_phase(p, d, b, i, pc);
        const int N = p.N[i], s0 = p.s0[i], k0 = p.k0[i];
        lin_fetch(B0, p, d, b, s0, k0, lane);  // the phase's first knot (its wait is in lin_knot)
        if (i > 0) { // dx_init = Px dX_end
            const double *Px = d.term + (b * p.P + (i - 1)) * TW + TM_PX;
            if (lane < NX) S.dx[lane] = dx;
            LSYNC();
            real a = 0;
            if (rowl)
                for (int j = 0; j < NX; ++j) a += (real)Px[r * NX + j] * S.dx[j];
            dx = a;
            LSYNC();
        } else {
            dx = 0;
        }
        if (rowl) {
            dx = dx + defg[(b * p.S + s0) * NX + r];
            if (st) d.dX[(b * p.S + s0) * NX + r] = dx;
        }
        // lxx row r (HKDCost.cpp:32): diagonal + foot cross terms
        LxxRow<real> lx_;
        lxx_row(p, pc, r, lx_);
        const real ru = rowl ? (real)(p.dt * r_diag(p, r)) : (real)0;
        // control r has a gain row only when its B column is non-zero (KCW layout)
        const bool stl = contact(pc, (rr % HC) / 3) != 0;
        const bool cpl = rowl && (rr < HC ? stl : !stl);
        const int krow0 = (rr % HC) * NX + cb;
        for (int k = 0; k < N; k += 2) {
            lin_knot(p, d, S, B0, B1, k + 1 < N, b, s0 + k, k0 + k, pc, lx_, ru, cpl, krow0, dx, v1, v2);
            if (k + 1 < N)
                lin_knot(p, d, S, B1, B0, k + 2 < N, b, s0 + k + 1, k0 + k + 1, pc, lx_, ru, cpl, krow0, dx, v1, v2);
        }
        const double *rec = d.term + (b * p.P + i) * TW;
        if (lane < NX) S.dx[lane] = dx;
        LSYNC();
        real q1 = 0, q2 = 0;
        if (rowl) {
            q1 = (real)rec[TM_PHIX + r] * dx;
            real a = 0;
            for (int c = 0; c < NX; ++c) a += (real)rec[TM_PHIXX + r * NX + c] * S.dx[c];
            q2 = dx * a;
        }
        v1 += half_sum(q1);
        v2 += half_sum(q2);
        LSYNC();
    }
    if (lane == 0) {
        const double cost = E.cost, feas = E.feas, w1 = v1, w2 = v2;
        const double dV_abs = fabs(w1 + 0.5 * w2);
        const double rho = (feas > p.feas_thresh) ? dV_abs / ((1 - p.merit_scale) * feas) + p.merit_offset : 0;
        const double merit = cost + rho * feas;
        E.dV1 = w1; E.dV2 = w2; E.merit_rho = rho; E.merit = merit;
        E.cost_prev = cost; E.merit_prev = merit; E.feas_prev = feas;
        if (!p.no_early_exit && dV_abs < p.cost_thresh && feas <= p.feas_thresh) { E.inner_done = 1; E.ls_active = 0; }
        else E.ls_active = 1;
    }
}

void launch_riccati(const Params &p, const Bufs &d, hipStream_t st)
{
    if (p.retry_cap > 0) (void)hipMemsetAsync(d.retry_count, 0, sizeof(int), st);
    if (p.fp32)
        hipLaunchKernelGGL(k_riccati<float>, dim3(p.B), dim3(64), 0, st, p, d);
    else
        hipLaunchKernelGGL(k_riccati<double>, dim3(p.B), dim3(64), 0, st, p, d);
    if (p.retry_cap > 0) {
        const dim3 gr((unsigned)(p.retry_cap * p.retry_m)), gs((unsigned)p.retry_cap);
        if (p.fp32) {
            hipLaunchKernelGGL(k_riccati_retry<float>, gr, dim3(64), 0, st, p, d);
            hipLaunchKernelGGL(k_riccati_select<float>, gs, dim3(64), 0, st, p, d);
        } else {
            hipLaunchKernelGGL(k_riccati_retry<double>, gr, dim3(64), 0, st, p, d);
            hipLaunchKernelGGL(k_riccati_select<double>, gs, dim3(64), 0, st, p, d);
        }
    }
}

void launch_lin_rollout(const Params &p, const Bufs &d, hipStream_t st)
{
    if (p.fp32)
        hipLaunchKernelGGL(k_lin_rollout<float>, dim3(p.B), dim3(64), 0, st, p, d);
    else
        hipLaunchKernelGGL(k_lin_rollout<double>, dim3(p.B), dim3(64), 0, st, p, d);
}

}  // namespace hsddp
