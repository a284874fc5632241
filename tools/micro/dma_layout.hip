// LDS-DMA stream probe for the linear rollout's access pattern: 2048
// single-wave workgroups, two "elements" per wave, each element reading one 4 KB image per "knot"
// for 200 knots, the next knot's images requested (global_load_lds_dwordx4) while the current one is
// consumed, double-buffered in LDS as k_lin_rollout does.  Two layouts of the same 3.4 GB:
//   element-major  [element][knot][4096 B]  (the solver's layout today)
//   knot-major     [knot][element][4096 B]  (the whole batch's knot k contiguous)
// with and without a stand-in for the per-knot compute (a dependent chain of multiply-adds on
// values read from the image).  Prints GB/s per variant.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/micro/dma_layout tools/micro/dma_layout.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int B = 4096, K = 200, IMG = 4096, NI = IMG / 1024;  // DMA instructions per element image

__device__ __forceinline__ void lds_dma16(const void *src, unsigned m0)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(m0)
                 : "memory");
}

template <bool KNOT_MAJOR>
__device__ __forceinline__ const char *image(const char *base, int e, int k)
{
    return base + (KNOT_MAJOR ? ((size_t)k * B + e) : ((size_t)e * K + k)) * IMG;
}

template <bool KNOT_MAJOR, int WORK>
__global__ __launch_bounds__(64, 2) void k_stream(const char *base, double *out)
{
    __shared__ __attribute__((aligned(16))) char buf[2][2][IMG];  // [buffer][element][bytes]
    const int lane = threadIdx.x, e0 = 2 * blockIdx.x;
    auto fetch = [&](int k, int nb) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < NI; ++j)
                lds_dma16(image<KNOT_MAJOR>(base, e0 + h, k) + 1024 * j + 16 * lane,
                          (unsigned)(size_t)(&buf[nb][h][1024 * j]));
    };
    double acc = lane;
    fetch(0, 0);
    for (int k = 0; k < K; ++k) {
        const int cb = k & 1;
        if (k + 1 < K) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the other buffer's reads are done
            fetch(k + 1, cb ^ 1);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");     // all but the 2 NI just issued
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const double *img = (const double *)buf[cb][lane >> 5];
        double v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = img[(lane & 31) + 32 * q];
#pragma unroll
        for (int r = 0; r < WORK; ++r)
#pragma unroll
            for (int q = 0; q < 8; ++q) acc = __builtin_fma(acc, v[q], 1e-3);
        if (WORK == 0) acc += v[0] + v[7];
    }
    out[blockIdx.x * 64 + lane] = acc;
}

template <bool KM, int W>
static double run(const char *base, double *out, hipEvent_t a, hipEvent_t b)
{
    hipLaunchKernelGGL((k_stream<KM, W>), dim3(B / 2), dim3(64), 0, 0, base, out);  // warm
    hipEventRecord(a);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k_stream<KM, W>), dim3(B / 2), dim3(64), 0, 0, base, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 3;
}

int main()
{
    const size_t bytes = (size_t)B * K * IMG;
    char *base = nullptr;
    double *out = nullptr;
    if (hipMalloc(&base, bytes) != hipSuccess || hipMalloc(&out, (size_t)B * 32 * sizeof(double)) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(base, 0, bytes);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    struct { const char *name; double ms; } r[4] = {
        {"element-major, no compute", run<false, 0>(base, out, a, b)},
        {"knot-major,    no compute", run<true, 0>(base, out, a, b)},
        {"element-major, 4x8 dependent FMAs per knot", run<false, 4>(base, out, a, b)},
        {"knot-major,    4x8 dependent FMAs per knot", run<true, 4>(base, out, a, b)},
    };
    for (auto &x : r) printf("%-45s %8.1f us  %7.2f TB/s\n", x.name, x.ms * 1e3, bytes / (x.ms * 1e-3) / 1e12);
    hipFree(base);
    hipFree(out);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
