// Stream probe for the linear rollout's per-knot traffic (k_lin_rollout): 2048 single-wave
// workgroups, two elements per wave, 200 knots, each knot's 4 KB image requested by LDS-DMA one knot
// ahead into a double buffer, as the kernel does.  Variants of where the image's bytes live and
// whether the knot also writes two 192-byte rows per element (dX, du):
//   one array      [element][knot][4096 B]                                  (the DMA probe)
//   four arrays    K [e][k][2304], LQ [e][k][1408], D [e][s][192], dU [e][k][192]  (the solver)
//   ... + writes   dX [e][s][192], du [e][k][192] stored one knot later (the solver)
//   one array + writes
// and with the image requests non-temporal (nt), the rows written as 4-knot runs or into knot-major arrays, and the stores' cache policy.  Prints the time and the read (+ write) rate per variant.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/micro/lin_streams tools/micro/lin_streams.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int B = 4096, K = 200, S = K + 4, IMG = 4096, NI = IMG / 1024;
constexpr int SK = 2304, SL = 1408, SD = 192, SU = 192;  // segment bytes of the solver's image

template <bool NT>
__device__ __forceinline__ void lds_dma16(const void *src, unsigned m0)
{
    unsigned keep;
    if constexpr (NT)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(src), "s"(m0)
                     : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(src), "s"(m0)
                     : "memory");
}

struct Arrays {
    const char *one, *k, *lq, *d, *du;
    double *wx, *wu;
};

// source of byte o (16-byte piece) of element e's knot k image
template <bool SPLIT>
__device__ __forceinline__ const char *src(const Arrays &a, int e, int k, int o)
{
    if constexpr (!SPLIT) return a.one + ((size_t)e * K + k) * IMG + o;
    if (o < SK) return a.k + ((size_t)e * K + k) * SK + o;
    o -= SK;
    if (o < SL) return a.lq + ((size_t)e * K + k) * SL + o;
    o -= SL;
    if (o < SD) return a.d + ((size_t)e * S + k + 1) * SD + o;
    o -= SD;
    return a.du + ((size_t)e * K + k) * SU + o;
}

// W: 0 no writes; 1 each knot's two rows stored one knot later (8 bytes per lane, the solver);
// 2 rows staged in LDS and stored every 4 knots as contiguous 768-byte runs (16 bytes per lane);
// 3 W = 1 without the image reads (writes only); 4 W = 1 into knot-major arrays [knot][element][24]
// store one double with cache policy POL: 0 default, 1 nt, 2 sc1, 3 sc0 sc1, 4 sc0
template <int POL>
__device__ __forceinline__ void st64(double *p, double v)
{
    if constexpr (POL == 0) *p = v;
    else if constexpr (POL == 1) asm volatile("global_store_dwordx2 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 2) asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 3) asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx2 %0, %1, off sc0" ::"v"(p), "v"(v) : "memory");
}

template <bool SPLIT, int W, bool NT, int POL = 0>
__global__ __launch_bounds__(64, 2) void k_stream(Arrays a, double *out)
{
    __shared__ __attribute__((aligned(16))) char buf[2][2][IMG];  // [buffer][element][bytes]
    __shared__ __attribute__((aligned(16))) double stg[2][2][4][24];  // [array][element][knot][row]
    const int lane = threadIdx.x, e0 = 2 * blockIdx.x, r = lane & 31, h = lane >> 5;
    auto fetch = [&](int k, int nb) {
        if constexpr (W == 3) return;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
            for (int j = 0; j < NI; ++j)
                lds_dma16<NT>(src<SPLIT>(a, e0 + hh, k, 1024 * j + 16 * lane), (unsigned)(size_t)(&buf[nb][hh][1024 * j]));
    };
    double acc = lane, px = 0, pu = 0;
    fetch(0, 0);
    for (int k = 0; k < K; ++k) {
        const int cb = k & 1;
        if (k + 1 < K) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            fetch(k + 1, cb ^ 1);
        }
        int ns = 0;
        if ((W == 1 || W == 3) && k > 0) {  // the previous knot's rows
            if (r < 24) {
                st64<POL>(a.wx + ((size_t)(e0 + h) * S + k) * 24 + r, px);
                st64<POL>(a.wu + ((size_t)(e0 + h) * K + k - 1) * 24 + r, pu);
            }
            ns = 2;
        }
        if (W == 4 && k > 0) {  // knot-major rows: [knot][element][24]
            if (r < 24) {
                a.wx[((size_t)k * B + e0 + h) * 24 + r] = px;
                a.wu[((size_t)(k - 1) * B + e0 + h) * 24 + r] = pu;
            }
            ns = 2;
        }
        if (W == 2 && k > 0 && (k & 3) == 0) {  // knots k - 4 .. k - 1: 2 arrays x 2 elements x 768 B
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            typedef double d2 __attribute__((ext_vector_type(2)));
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int f = lane + 64 * t;  // 16-byte piece of 192
                if (f < 192) {
                    const int arr = f / 96, e = (f / 48) & 1, q = f % 48;
                    const d2 v = ((const d2 *)&stg[arr][e][0][0])[q];
                    double *dst = arr ? a.wu + ((size_t)(e0 + e) * K + k - 4) * 24 : a.wx + ((size_t)(e0 + e) * S + k - 3) * 24;
                    ((d2 *)dst)[q] = v;
                }
            }
            ns = 3;
        }
        if (k + 1 < K && W != 3) {
            if (ns == 2) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
            else if (ns == 3) asm volatile("s_waitcnt vmcnt(11)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else if (W != 3) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const double *img = (const double *)buf[cb][h];
        double v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = img[r + 32 * q];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int q = 0; q < 8; ++q) acc = __builtin_fma(acc, v[q], 1e-3);
        px = acc;
        pu = acc + v[1];
        if (W == 2 && r < 24) {
            stg[0][h][k & 3][r] = px;
            stg[1][h][k & 3][r] = pu;
        }
    }
    out[blockIdx.x * 64 + lane] = acc;
}

template <bool SP, int W, bool NT, int POL = 0>
static double run(const Arrays &a, double *out, hipEvent_t e0, hipEvent_t e1)
{
    hipLaunchKernelGGL((k_stream<SP, W, NT, POL>), dim3(B / 2), dim3(64), 0, 0, a, out);  // warm
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k_stream<SP, W, NT, POL>), dim3(B / 2), dim3(64), 0, 0, a, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main()
{
    const size_t one = (size_t)B * K * IMG, nk = (size_t)B * K * SK, nl = (size_t)B * K * SL, nd = (size_t)B * S * SD,
                 nu = (size_t)B * K * SU, nwx = (size_t)B * S * 24 * 8, nwu = (size_t)B * K * 24 * 8;
    char *p[7] = {};
    size_t sz[7] = {one, nk, nl, nd, nu, nwx, nwu};
    for (int i = 0; i < 7; ++i)
        if (hipMalloc(&p[i], sz[i]) != hipSuccess || hipMemset(p[i], 0, sz[i]) != hipSuccess) {
            printf("alloc failed\n");
            return 1;
        }
    double *out = nullptr;
    if (hipMalloc(&out, (size_t)B * 32 * sizeof(double)) != hipSuccess) return 1;
    Arrays a{p[0], p[1], p[2], p[3], p[4], (double *)p[5], (double *)p[6]};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double rd = (double)B * K * IMG, wr = (double)B * K * 2 * 192;
    struct { const char *name; double ms, bytes; } r[] = {
        {"one array", run<false, 0, false>(a, out, e0, e1), rd},
        {"four arrays", run<true, 0, false>(a, out, e0, e1), rd},
        {"one array + writes", run<false, 1, false>(a, out, e0, e1), rd + wr},
        {"four arrays + writes", run<true, 1, false>(a, out, e0, e1), rd + wr},
        {"one array nt", run<false, 0, true>(a, out, e0, e1), rd},
        {"one array nt + writes", run<false, 1, true>(a, out, e0, e1), rd + wr},
        {"four arrays nt + writes", run<true, 1, true>(a, out, e0, e1), rd + wr},
        {"one array + 4-knot writes", run<false, 2, false>(a, out, e0, e1), rd + wr},
        {"one array nt + 4-knot writes", run<false, 2, true>(a, out, e0, e1), rd + wr},
        {"writes only", run<false, 3, false>(a, out, e0, e1), wr},
        {"one array + knot-major writes", run<false, 4, false>(a, out, e0, e1), rd + wr},
        {"one array nt + knot-major writes", run<false, 4, true>(a, out, e0, e1), rd + wr},
        {"four arrays nt + knot-major writes", run<true, 4, true>(a, out, e0, e1), rd + wr},
        {"four arrays nt + writes nt", run<true, 1, true, 1>(a, out, e0, e1), rd + wr},
        {"four arrays nt + writes sc1", run<true, 1, true, 2>(a, out, e0, e1), rd + wr},
        {"four arrays nt + writes sc0 sc1", run<true, 1, true, 3>(a, out, e0, e1), rd + wr},
        {"four arrays nt + writes sc0", run<true, 1, true, 4>(a, out, e0, e1), rd + wr},
        {"four arrays + writes nt", run<true, 1, false, 1>(a, out, e0, e1), rd + wr},
    };
    for (auto &x : r) printf("%-30s %8.1f us  %7.2f TB/s (reads + writes)\n", x.name, x.ms * 1e3, x.bytes / (x.ms * 1e-3) / 1e12);
    for (int i = 0; i < 7; ++i) hipFree(p[i]);
    hipFree(out);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
