// Issue-rate probes for gfx950 (fp64 VALU, v_readlane, f64 MFMA, VALU+MFMA mix).  Each kernel runs
// ITER iterations of an unrolled body on every wave of a full grid; rates are printed per CU per
// cycle at the measured shader clock (s_memtime deltas vs event time).
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITER = 4096;
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void k_fma(double *out, double s)
{
    double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_fma_f64 %0, %0, %8, %8\n\tv_fma_f64 %1, %1, %8, %8\n\tv_fma_f64 %2, %2, %8, %8\n\tv_fma_f64 %3, %3, %8, %8\n\t"
                     "v_fma_f64 %4, %4, %8, %8\n\tv_fma_f64 %5, %5, %8, %8\n\tv_fma_f64 %6, %6, %8, %8\n\tv_fma_f64 %7, %7, %8, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(s));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// v_fmac_f64 with a DPP row_newbcast source (the sweep's broadcast-coefficient form)
__global__ void k_fma_dpp(double *out, double s)
{
    double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    double c = s * threadIdx.x;
    asm volatile("s_nop 4" ::: "memory");
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_fmac_f64_dpp %0, %8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %1, %8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %2, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %3, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %4, %8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %5, %8, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %6, %8, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %7, %8, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(c), "v"(s));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

__global__ void k_add32(double *out, double s)
{
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    unsigned t = (unsigned)s;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
                     "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(t));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

__global__ void k_readlane(double *out, double s)
{
    unsigned v = threadIdx.x * 3 + (unsigned)s;
    unsigned x0 = 0, x1 = 0, x2 = 0, x3 = 0, x4 = 0, x5 = 0, x6 = 0, x7 = 0;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_readlane_b32 %0, %8, 1\n\tv_readlane_b32 %1, %8, 2\n\tv_readlane_b32 %2, %8, 3\n\tv_readlane_b32 %3, %8, 4\n\t"
                     "v_readlane_b32 %4, %8, 5\n\tv_readlane_b32 %5, %8, 6\n\tv_readlane_b32 %6, %8, 7\n\tv_readlane_b32 %7, %8, 8"
                     : "=s"(x0), "=s"(x1), "=s"(x2), "=s"(x3), "=s"(x4), "=s"(x5), "=s"(x6), "=s"(x7)
                     : "v"(v));
        v += x0 ^ x7;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = v + x1 + x2 + x3 + x4 + x5 + x6;
}

__global__ void k_mfma(double *out, double s)
{
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    double a = threadIdx.x * s, b = s;
    for (int i = 0; i < ITER / 4; ++i) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    d4 c = c0 + c1 + c2 + c3;
    out[blockIdx.x * blockDim.x + threadIdx.x] = c[0] + c[1] + c[2] + c[3];
}

// half the waves MFMA, half VALU fma (same kernel, branch on wave id): concurrency check
__global__ void k_mix(double *out, double s)
{
    if ((threadIdx.x >> 6) & 1) {
        d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
        double a = threadIdx.x * s, b = s;
        for (int i = 0; i < ITER / 4; ++i) {
            c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
        }
        d4 c = c0 + c1 + c2 + c3;
        out[blockIdx.x * blockDim.x + threadIdx.x] = c[0] + c[1] + c[2] + c[3];
    } else {
        double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
        for (int i = 0; i < ITER; ++i) {
            asm volatile("v_fma_f64 %0, %0, %8, %8\n\tv_fma_f64 %1, %1, %8, %8\n\tv_fma_f64 %2, %2, %8, %8\n\tv_fma_f64 %3, %3, %8, %8\n\t"
                         "v_fma_f64 %4, %4, %8, %8\n\tv_fma_f64 %5, %5, %8, %8\n\tv_fma_f64 %6, %6, %8, %8\n\tv_fma_f64 %7, %7, %8, %8"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(s));
        }
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    }
}

__global__ void k_lds(double *out, double s)
{
    __shared__ double L[1024];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) L[i] = i * s;
    __syncthreads();
    double acc = 0;
    int base = (threadIdx.x >> 6) * 16;
    for (int i = 0; i < ITER / 8; ++i) {
        typedef double d2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            d2 v = *(volatile d2 *)&L[(base + 2 * j + i) & 1023];
            acc += v[0] * v[1];
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <typename K>
float run(K k, int blocks, int threads, double *out)
{
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 1.0000001);
    hipEventRecord(a);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 1.0000001);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main()
{
    hipDeviceProp_t pr; hipGetDeviceProperties(&pr, 0);
    const int cu = pr.multiProcessorCount;
    const double ghz = pr.clockRate / 1e6;
    double *out; hipMalloc(&out, 1 << 26);
    printf("CUs %d clock %.3f GHz\n", cu, ghz);
    for (int wps : {4, 8, 16}) {  // waves per CU (256-thread blocks = 4 waves)
        int blocks = cu * wps / 4 * 8;  // 8 rounds
        double waves = blocks * 4.0;
        float ms;
        ms = run(k_fma, blocks, 256, out);
        printf("wpcu %2d fma_f64   : %.2f wave-instr/cycle/CU  (%.1f TF)\n", wps, waves * ITER * 8 / (ms * 1e-3 * ghz * 1e9) / cu,
               waves * 64 * ITER * 8 * 2 / (ms * 1e-3) / 1e12);
        ms = run(k_fma_dpp, blocks, 256, out);
        printf("wpcu %2d fma_f64_dpp: %.2f wave-instr/cycle/CU  (%.1f TF)\n", wps, waves * ITER * 8 / (ms * 1e-3 * ghz * 1e9) / cu,
               waves * 64 * ITER * 8 * 2 / (ms * 1e-3) / 1e12);
        ms = run(k_add32, blocks, 256, out);
        printf("wpcu %2d add_u32   : %.2f wave-instr/cycle/CU\n", wps, waves * ITER * 8 / (ms * 1e-3 * ghz * 1e9) / cu);
        ms = run(k_readlane, blocks, 256, out);
        printf("wpcu %2d readlane  : %.2f wave-instr/cycle/CU\n", wps, waves * ITER * 8 / (ms * 1e-3 * ghz * 1e9) / cu);
        ms = run(k_mfma, blocks, 256, out);
        printf("wpcu %2d mfma_f64  : %.3f wave-instr/cycle/CU (%.1f TF)\n", wps, waves * ITER / (ms * 1e-3 * ghz * 1e9) / cu,
               waves * ITER * 1024.0 * 2 / (ms * 1e-3) / 1e12);
        ms = run(k_mix, blocks, 256, out);
        printf("wpcu %2d mix       : %.3f ms  (fma-only equiv %.3f, mfma-only equiv %.3f)\n", wps, ms,
               run(k_fma, blocks / 2, 256, out), run(k_mfma, blocks / 2, 256, out));
        ms = run(k_lds, blocks, 256, out);
        printf("wpcu %2d ds_read128: %.2f wave-instr/cycle/CU\n", wps, waves * ITER / (ms * 1e-3 * ghz * 1e9) / cu);
    }
    return 0;
}
