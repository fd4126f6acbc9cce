// Throughput of individual f64 VALU instructions on gfx950 (8 independent
// chains per lane, 1024 blocks x 256 threads).  Reports cycles per wave-
// instruction per SIMD at the measured clock-free ratio to v_fma_f64.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_ops.hip -o tools/ubench_ops
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAINS 8
template <int OP> __device__ __forceinline__ double op(double x, double s, int i)
{
    if (OP == 0) return fma(x, s, 0.5);
    if (OP == 1) return x + s;
    if (OP == 2) return x * s;
    if (OP == 3) return __builtin_rint(x * s);          // mul + rndne (2 ops)
    if (OP == 4) return (double)(int)(x) + s;           // cvt_i32 + cvt_f64 + add
    if (OP == 5) return __builtin_ldexp(x, i);          // ldexp
    if (OP == 6) return fmax(x, s);
    return x;
}

template <int OP> __global__ __launch_bounds__(256) void kern(double *out, int iters, double s)
{
    double v[CHAINS];
    for (int c = 0; c < CHAINS; ++c) v[c] = threadIdx.x * 1e-3 + c;
    int sh = (threadIdx.x & 1) ? 1 : -1;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int q = 0; q < 8; ++q)
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) v[c] = op<OP>(v[c], s, sh);
    }
    double r = 0;
    for (int c = 0; c < CHAINS; ++c) r += v[c];
    if (r == 1234.5678) out[threadIdx.x] = r;
}

template <int OP> float run(int blocks, int iters)
{
    double *out;
    (void)hipMalloc(&out, 4096);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    kern<OP><<<blocks, 256>>>(out, 10, 0.9999);
    (void)hipEventRecord(e0);
    kern<OP><<<blocks, 256>>>(out, iters, 0.9999);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(out);
    return ms;
}

int main()
{
    const int blocks = 1024, iters = 2000;
    const char *names[] = {"fma", "add", "mul", "mul+rndne", "cvt_i32+cvt_f64+add", "ldexp", "max"};
    float t[7];
    t[0] = run<0>(blocks, iters);
    t[1] = run<1>(blocks, iters);
    t[2] = run<2>(blocks, iters);
    t[3] = run<3>(blocks, iters);
    t[4] = run<4>(blocks, iters);
    t[5] = run<5>(blocks, iters);
    t[6] = run<6>(blocks, iters);
    const double ops = (double)blocks * 4 * iters * 8 * CHAINS; // wave-instructions per op slot
    for (int i = 0; i < 7; ++i)
        printf("%-22s %8.3f ms  %.3f x fma time  (%.2f Gwave-instr/s)\n", names[i], t[i], t[i] / t[0],
               ops / t[i] / 1e6);
    return 0;
}
