// Does v_lshlrev_b16 zero the high 16 bits of its 32-bit destination on
// gfx950 (legacy gfx9 behaviour)?  The phi row stream's 8192-entry exp table
// address relies on it ((ki << 3) & 0xffff in one instruction).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const int *in, unsigned *out)
{
    const int ki = in[threadIdx.x];
    unsigned r = 0xdeadbeefu;
    asm volatile("v_mov_b32 %0, 0xdeadbeef\n\tv_lshlrev_b16 %0, 3, %1" : "+v"(r) : "v"(ki));
    out[threadIdx.x] = r;
}
int main()
{
    int h[64];
    for (int i = 0; i < 64; ++i) h[i] = (i * 1234567 - 40000000) ^ (i << 20);
    int *din;
    unsigned *dout, hout[64];
    (void)hipMalloc(&din, sizeof h);
    (void)hipMalloc(&dout, sizeof hout);
    (void)hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout);
    (void)hipMemcpy(hout, dout, sizeof hout, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 64; ++i)
        if (hout[i] != (((unsigned)h[i] << 3) & 0xffffu)) ++bad;
    printf("v_lshlrev_b16 zeroes the high bits: %s (%d mismatches; e.g. in %08x -> %08x)\n",
           bad ? "NO" : "yes", bad, (unsigned)h[5], hout[5]);
    return bad ? 1 : 0;
}
