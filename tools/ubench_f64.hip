// Micro-benchmark: do MFMA and VALU work of the same precision run concurrently
// on gfx950?  Decides whether the fp64 phi / median kernels should put their
// dot products and contractions on the matrix cores.
//
// Variants (1024 blocks x 256 threads = 4 waves per SIMD):
//   mfma only / valu only        -- each pipe alone
//   mixed (same wave)            -- MFMAs and independent FMAs interleaved in one stream
//   split by block               -- even blocks MFMA-only, odd blocks VALU-only, so every
//                                   SIMD holds MFMA waves beside VALU waves
// for f64 (v_mfma_f64_16x16x4f64 + v_fma_f64) and f32 (v_mfma_f32_16x16x4f32 + v_fma_f32).
// "total" = MFMA + VALU flop rate; pipes that overlap show total ~ sum of the two alone.
//
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_f64.hip -o tools/ubench_f64
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <class T> struct MF;
template <> struct MF<double> {
    typedef d4 V;
    static __device__ __forceinline__ V op(double a, double b, V c)
    {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
};
template <> struct MF<float> {
    typedef f4 V;
    static __device__ __forceinline__ V op(float a, float b, V c)
    {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
};

// MODE 0: mfma only, 1: valu only, 2: mixed in one wave, 3: split by block parity
template <class T, int MODE, int NM, int NV>
__global__ __launch_bounds__(256) void kern(T *out, int iters, T s)
{
    typedef typename MF<T>::V V;
    V acc0 = {0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
    T a = threadIdx.x * (T)1e-3, b = s;
    T v0 = a, v1 = a + 1, v2 = a + 2, v3 = a + 3, v4 = a + 4, v5 = a + 5, v6 = a + 6, v7 = a + 7;
    const bool do_m = MODE == 0 || MODE == 2 || (MODE == 3 && (blockIdx.x & 1) == 0);
    const bool do_v = MODE == 1 || MODE == 2 || (MODE == 3 && (blockIdx.x & 1) == 1);
    if (do_m && !do_v) {
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int m = 0; m < NM / 4; ++m) {
                acc0 = MF<T>::op(a, b, acc0);
                acc1 = MF<T>::op(a, b, acc1);
                acc2 = MF<T>::op(a, b, acc2);
                acc3 = MF<T>::op(a, b, acc3);
            }
        }
    } else if (do_v && !do_m) {
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int q = 0; q < NV / 8; ++q) {
                v0 = fma(v0, s, b); v1 = fma(v1, s, b); v2 = fma(v2, s, b); v3 = fma(v3, s, b);
                v4 = fma(v4, s, b); v5 = fma(v5, s, b); v6 = fma(v6, s, b); v7 = fma(v7, s, b);
            }
        }
    } else {
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int m = 0; m < NM / 4; ++m) {
                acc0 = MF<T>::op(a, b, acc0);
                acc1 = MF<T>::op(a, b, acc1);
                acc2 = MF<T>::op(a, b, acc2);
                acc3 = MF<T>::op(a, b, acc3);
#pragma unroll
                for (int q = 0; q < NV / NM / 2; ++q) {
                    v0 = fma(v0, s, b); v1 = fma(v1, s, b); v2 = fma(v2, s, b); v3 = fma(v3, s, b);
                    v4 = fma(v4, s, b); v5 = fma(v5, s, b); v6 = fma(v6, s, b); v7 = fma(v7, s, b);
                }
            }
        }
    }
    T r = acc0[0] + acc1[1] + acc2[2] + acc3[3] + v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;
    if (r == (T)12345.678) out[threadIdx.x] = r;
}

template <class T, int MODE, int NM, int NV> void run(const char *name)
{
    const int blocks = 1024, iters = 4000;
    T *out;
    (void)hipMalloc(&out, 4096);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    kern<T, MODE, NM, NV><<<blocks, 256>>>(out, 20, (T)0.999);
    (void)hipEventRecord(e0);
    kern<T, MODE, NM, NV><<<blocks, 256>>>(out, iters, (T)0.999);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double waves = blocks * 4.0;
    const double mw = MODE == 1 ? 0 : MODE == 3 ? waves / 2 : waves;
    const double vw = MODE == 0 ? 0 : MODE == 3 ? waves / 2 : waves;
    const double mfma_flops = mw * iters * NM * 2048.0;
    const double valu_flops = vw * iters * NV * 64 * 2.0; // NV fma per lane per iteration
    printf("%-4s %-34s %8.3f ms  MFMA %6.1f TF  VALU %6.1f TF  total %6.1f TF\n",
           sizeof(T) == 8 ? "f64" : "f32", name, ms, mfma_flops / ms / 1e9, valu_flops / ms / 1e9,
           (mfma_flops + valu_flops) / ms / 1e9);
    (void)hipFree(out);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

template <class T> void suite()
{
    run<T, 0, 16, 0>("mfma only (16 per iter)");
    run<T, 1, 0, 64>("valu only (64 fma per iter)");
    run<T, 2, 16, 64>("mixed in one wave: 16 mfma + 64 fma");
    run<T, 2, 16, 128>("mixed in one wave: 16 mfma + 128 fma");
    run<T, 3, 16, 64>("split by block: mfma | valu waves");
}

int main()
{
    suite<double>();
    suite<float>();
    return 0;
}
