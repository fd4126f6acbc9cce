// Micro-benchmark: can f64 MFMA (v_mfma_f64_16x16x4_f64) and f64 VALU
// (v_fma_f64) run concurrently on gfx950?  Prints cycles-equivalent rates.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_f64.hip -o /tmp/ubench_f64
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int NM, int NV>
__global__ __launch_bounds__(256) void kern(double *out, int iters, double s)
{
    d4 acc0 = {0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
    double a = threadIdx.x * 1e-3, b = s;
    double v0 = a, v1 = a + 1, v2 = a + 2, v3 = a + 3, v4 = a + 4, v5 = a + 5, v6 = a + 6, v7 = a + 7;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            if (m % 4 == 0) acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
            if (m % 4 == 1) acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc1, 0, 0, 0);
            if (m % 4 == 2) acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc2, 0, 0, 0);
            if (m % 4 == 3) acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc3, 0, 0, 0);
#pragma unroll
            for (int q = 0; q < NV / (NM ? NM : 1); ++q) {
                v0 = fma(v0, s, b); v1 = fma(v1, s, b); v2 = fma(v2, s, b); v3 = fma(v3, s, b);
                v4 = fma(v4, s, b); v5 = fma(v5, s, b); v6 = fma(v6, s, b); v7 = fma(v7, s, b);
            }
        }
        if (NM == 0) {
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                v0 = fma(v0, s, b); v1 = fma(v1, s, b); v2 = fma(v2, s, b); v3 = fma(v3, s, b);
                v4 = fma(v4, s, b); v5 = fma(v5, s, b); v6 = fma(v6, s, b); v7 = fma(v7, s, b);
            }
        }
    }
    double r = acc0[0] + acc1[1] + acc2[2] + acc3[3] + v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;
    if (r == 12345.678) out[threadIdx.x] = r;
}

template <int NM, int NV> void run(const char *name, int blocks)
{
    double *out;
    hipMalloc(&out, 4096);
    const int iters = 2000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    kern<NM, NV><<<blocks, 256>>>(out, 10, 0.999);
    hipEventRecord(e0);
    kern<NM, NV><<<blocks, 256>>>(out, iters, 0.999);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double waves = blocks * 4.0;
    double mfma_flops = waves * iters * NM * 2048.0;
    double valu_flops = waves * iters * (NM ? (NV / NM) * NM : NV) * 8 * 64 * 2.0;
    printf("%-28s blocks=%5d  %8.3f ms  MFMA %6.1f TF  VALU %6.1f TF  total %6.1f TF\n", name, blocks,
           ms, mfma_flops / ms / 1e9, valu_flops / ms / 1e9, (mfma_flops + valu_flops) / ms / 1e9);
    hipFree(out);
}

int main()
{
    for (int blocks : {256, 1024}) {
        run<16, 0>("mfma only (16/iter)", blocks);
        run<0, 8>("valu only (64 fma/iter)", blocks);
        run<16, 16>("mfma16 + valu128", blocks);
        run<16, 32>("mfma16 + valu256", blocks);
        run<16, 64>("mfma16 + valu512", blocks);
    }
    return 0;
}
