// svgd_kernels.hip -- CDNA4 (gfx950) kernels of the SVGD inner step.
//
// Reference hot path (khaiyichin/SVGDCpp, paths relative to its root):
//   GaussianRBFKernel::ComputeScale (Median) + ComputeMedian
//       include/SVGDCpp/Kernel/GaussianRBFKernel.hpp:164-188, 222-254
//   SVGD::ComputePhi (K, Kg, (1/N)(G K + [I..I] Kg))   include/SVGDCpp/SVGD.hpp:407-454
//   RBF lambda exp(-(x-x')^T M (x-x'))                 GaussianRBFKernel.hpp:75-81
//   Adam / AdaGrad / RMSProp Step                       Optimizer/*.hpp
//   X += Step(phi); clamp                               SVGD.hpp:393-399
//
// Device data layout (HBM): particle-major, i.e. the reference's d x n
// column-major Eigen matrix: particle j at X[j*d .. j*d+d-1].  The working
// copies are padded: xc[j*KP + k] holds the mean-centred coordinates with
// k padded to KP (multiple of 4, the f64 MFMA K), V[j*16*NCB + c] holds
// [G_j - 2a xc_j, 1, 0 ...] (the phi contraction operand), rows padded to a
// multiple of 64 with zeros.
//
// f64 MFMA: v_mfma_f64_16x16x4_f64.  A/B lane maps: A[i = l&15][k = l>>4],
// B[k = l>>4][j = l&15]; C/D: col = l&15, row = (l>>4) + 4*reg.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <type_traits>
#include <stdint.h>

#include "svgd_kernels.h"
#include "svgd_exp_table.h"
#include "svgd_device.h"

namespace svgd_amd {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int LDP = TB + 16; // padded LDS row stride (doubles) of the k-major X tiles

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ d4 mfma64(double a, double b, d4 c)
{
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// Same 16x16x4 lane maps for both precisions (the fp32 path, SVGD_F32, runs
// the tile kernels on v_mfma_f32_16x16x4f32).
template <class T> struct Acc4;
template <> struct Acc4<double> {
    typedef d4 type;
};
template <> struct Acc4<float> {
    typedef f4 type;
};
__device__ __forceinline__ d4 mfma16(double a, double b, d4 c)
{
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f4 mfma16(float a, float b, f4 c)
{
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// Row of accumulator register r in lane group hi = lane >> 4 (column = lane & 15):
// f64 16x16x4 interleaves the groups (row = hi + 4r), f32 16x16x4 gives each
// group 4 consecutive rows (row = 4hi + r).  A/B maps are the same for both.
template <class T> __device__ __forceinline__ int acc_row(int hi, int r);
template <> __device__ __forceinline__ int acc_row<double>(int hi, int r) { return hi + 4 * r; }
template <> __device__ __forceinline__ int acc_row<float>(int hi, int r) { return 4 * hi + r; }

// 2^t for t <= 0 (t = -a*log2(e)*s).  Range reduction t = k + f, |f| <= 1/2,
// degree-12 Taylor polynomial of 2^f (max error 1.9 ulp on [-1/2, 1/2]),
// v_ldexp_f64 for 2^k.  Results below 2^-1075 flush to 0 like exp() does.
__device__ __forceinline__ double exp2_neg(double t)
{
    t = fmax(t, -1075.0);
    const double k = __builtin_rint(t);
    const double f = t - k;
    double p = 0x1.c3bd650fc2986p-36;
    p = fma(p, f, 0x1.e8cac7351bb25p-32);
    p = fma(p, f, 0x1.e4cf5158b8ecap-28);
    p = fma(p, f, 0x1.b5253d395e7c4p-24);
    p = fma(p, f, 0x1.62c0223a5c824p-20);
    p = fma(p, f, 0x1.ffcbfc588b0c7p-17);
    p = fma(p, f, 0x1.430912f86c787p-13);
    p = fma(p, f, 0x1.5d87fe78a6731p-10);
    p = fma(p, f, 0x1.3b2ab6fba4e77p-7);
    p = fma(p, f, 0x1.c6b08d704a0c0p-5);
    p = fma(p, f, 0x1.ebfbdff82c58fp-3);
    p = fma(p, f, 0x1.62e42fefa39efp-1);
    p = fma(p, f, 1.0);
    return __builtin_ldexp(p, (int)k);
}

constexpr double LOG2E = 0x1.71547652b82fep+0;

// 2^t for t <= 0 in the tile kernels' precision (fp32: v_exp_f32, 1 ulp)
__device__ __forceinline__ double exp2_nonpos(double t) { return exp2_neg(fmin(t, 0.0)); }
__device__ __forceinline__ float exp2_nonpos(float t) { return __builtin_amdgcn_exp2f(fminf(t, 0.0f)); }

// fp32 working copies for the SVGD_F32 path (rows of padded arrays)
__global__ void k_cvt_f32(const double *__restrict__ src, int64_t cnt, float *__restrict__ dst)
{
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < cnt;
         e += (int64_t)gridDim.x * blockDim.x)
        dst[e] = (float)src[e];
}

// ------------------------------------------------------------ centering --

// Per-block partial column sums of X (n x d) -> partial[b*d + k].  Block b
// sums a contiguous run of whole rows; thread t reads elements t, t + ST, ...
// (ST = the largest multiple of d <= 256, so a thread always sees the same
// column k = t mod d: coalesced loads), then the threads of each column are
// summed in fixed order (deterministic).
__global__ void k_mean_partial(const double *__restrict__ X, int64_t n, int d,
                               double *__restrict__ partial, unsigned long long *nmax_bits)
{
    __shared__ double red[256];
    if (nmax_bits && blockIdx.x == 0 && threadIdx.x == 0) *nmax_bits = 0; // k_center's atomicMax target
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t j0 = per * blockIdx.x, j1 = min(n, j0 + per);
    const int ST = d <= 256 ? 256 - 256 % d : 0;
    const int t = threadIdx.x;
    double s = 0.0;
    if (ST > 0 && t < ST && j1 > j0) {
        const int64_t e1 = j1 * d;
        for (int64_t e0 = j0 * d + t; e0 < e1; e0 += 8 * ST) {
            double v[8]; // 8 loads in flight, added in order
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = e0 + u * ST < e1 ? X[e0 + u * ST] : 0.0;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (e0 + u * ST < e1) s += v[u];
        }
    }
    red[t] = s;
    __syncthreads();
    if (ST > 0) {
        if (t < d) {
            double c = 0.0;
            for (int u = t; u < ST; u += d) c += red[u];
            partial[blockIdx.x * d + t] = c;
        }
    } else {
        // d > 256: one column at a time (rare; not a hot configuration)
        for (int k = 0; k < d; ++k) {
            __syncthreads();
            double c = 0.0;
            for (int64_t j = j0 + t; j < j1; j += blockDim.x) c += X[j * d + k];
            red[t] = c;
            __syncthreads();
            if (t == 0) {
                double q = 0.0;
                for (int u = 0; u < 256; ++u) q += red[u];
                partial[blockIdx.x * d + k] = q;
            }
        }
    }
}

// xc = X - mean (padded to KP columns, rows [n, np) zero), nrm = |xc|^2.
// The mean is re-derived by every block from the partials in a fixed order,
// so it is bit-identical on every rank and block.
// With xf: also the fp32 median record [fl(xc) | fl(-|xc|^2/2) | 0..] (stride
// KF = med_f32_stride(d)) and max_j |xc_j|^2 into *nmax_bits (non-negative
// doubles order like their bit patterns).
__global__ void k_center(const double *__restrict__ X, int64_t n, int d, int KP,
                         const double *__restrict__ partial, int nparts, int64_t np,
                         double *__restrict__ xc, double *__restrict__ nrm, int nrm_in_slot,
                         float *__restrict__ xf, int KF, unsigned long long *nmax_bits,
                         unsigned long long *bzero, SelState *st_out, SelState st_init)
{
    if (bzero && blockIdx.x == 0) // this step's collect-pass bucket counts
        for (int e = threadIdx.x; e < NBK; e += blockDim.x) bzero[e] = 0;
    if (st_out && blockIdx.x == 0 && threadIdx.x == 0) *st_out = st_init; // predicted bracket
    __shared__ double mu[256];
    for (int k = threadIdx.x; k < d; k += blockDim.x) {
        // partials added in b order; 8 loads in flight
        double s = 0.0;
        for (int b0 = 0; b0 < nparts; b0 += 8) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = b0 + u < nparts ? partial[(b0 + u) * d + k] : 0.0;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (b0 + u < nparts) s += v[u];
        }
        mu[k] = s / (double)n;
    }
    __syncthreads();
    unsigned long long bmax = 0;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < np;
         j += (int64_t)gridDim.x * blockDim.x) {
        double s = 0.0;
        for (int k = 0; k < KP; ++k) {
            double v = (j < n && k < d) ? X[j * d + k] - mu[k] : 0.0;
            xc[j * KP + k] = v;
            s = fma(v, v, s);
        }
        nrm[j] = s;
        if (KP > d && nrm_in_slot) xc[j * KP + d] = -0.5 * s; // median record [xc | -|xc|^2/2 | 0..]
        if (xf) {
            // padding rows j >= n: h = -inf (k_pair_mcol reads whole 16-column blocks)
            for (int k = 0; k < KF; ++k)
                xf[j * KF + k] = k < d ? (float)xc[j * KP + k]
                                       : (k == d ? (j < n ? (float)(-0.5 * s) : -__builtin_inff()) : 0.0f);
            unsigned long long m = (unsigned long long)__double_as_longlong(s);
            for (int o = 32; o > 0; o >>= 1) {
                const unsigned long long t = __shfl_xor(m, o);
                m = t > m ? t : m;
            }
            bmax = m > bmax ? m : bmax;
        }
    }
    if (xf) {
        // one atomic per block (per-wave atomics on one address serialise)
        __shared__ unsigned long long wmax[4];
        if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = bmax;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long m = 0;
            for (int w = 0; w < (int)(blockDim.x >> 6); ++w) m = wmax[w] > m ? wmax[w] : m;
            atomicMax(nmax_bits, m);
        }
    }
}

// The centre of a centring from `nin` column-sum partials (nin * D <= 4096,
// staged in sP): mu[k] = (sum of the partials) / n, every block summing them
// in the same fixed order -- T threads per column take partials q, q + T, ...
// in turn, then their T sums meet in a fixed tree -- so the centre is
// bit-identical in every block and on every rank.
template <int D>
__device__ __forceinline__ void center_mean(const double *__restrict__ pin, int nin, int64_t n, double *sP,
                                            double *mu)
{
    constexpr int T = D <= 2 ? 128 : D <= 4 ? 64 : D <= 8 ? 32 : 16; // threads per column
    for (int e = threadIdx.x; e < nin * D; e += blockDim.x) sP[e] = pin[e];
    __syncthreads();
    __shared__ double sT[D <= 2 ? 64 * D : 1];
    const int k = threadIdx.x / T, q = threadIdx.x - k * T;
    double s = 0.0;
    if (k < D)
        for (int b = q; b < nin; b += T) s += sP[b * D + k];
    // the T sums in a fixed tree: partner q + h for h = T/2 .. 1 (T = 128:
    // the upper wave's sums through LDS first, then within the wave by
    // shuffles -- a column's T <= 64 threads are one aligned lane group)
    if constexpr (T == 128) {
        if (k < D && q >= 64) sT[k * 64 + q - 64] = s;
        __syncthreads();
        if (k < D && q < 64) s += sT[k * 64 + q];
    }
#pragma unroll
    for (int h = (T > 64 ? 64 : T) / 2; h > 0; h >>= 1) s += __shfl_xor(s, h);
    if (k < D && q == 0) mu[k] = s / (double)n;
    __syncthreads();
}

// k_center for d <= 16 with the median record stride KP = med_rec_stride(D):
// xc = X - mu, |xc|^2, the median records, max |xc|^2, with the row's X
// loads unrolled and issued before the centre is formed (one row ahead: the
// generic loop was latency-bound at 20 us for N = 65536, d = 8) and 16-byte
// record stores.  The centre mu is the mean of the partials `pin`: those of
// k_mean_partial (the exact mean of this X), or -- one launch per step --
// those this kernel left for the previous X (its mean: any fixed centre near
// the particles keeps the centred Gram form accurate, and the distances and
// kernel values are translation invariant).  pout: this block's column sums
// of its rows of X (the next centring's partials, gridDim.x * D values).
// nmax_zero: the other max |xc|^2 slot, zeroed for the next centring.
template <int D>
__global__ __launch_bounds__(256) void k_center_d(const double *__restrict__ X, int64_t n,
                                                  const double *__restrict__ pin, int nin,
                                                  int64_t np, double *__restrict__ xc,
                                                  double *__restrict__ nrm, int nrm_in_slot,
                                                  float *__restrict__ xf,
                                                  unsigned long long *nmax_bits,
                                                  unsigned long long *nmax_zero, double *__restrict__ pout,
                                                  unsigned long long *bzero, SelState *st_out,
                                                  SelState st_init, uint4 *__restrict__ xs)
{
    constexpr int KP = med_rec_stride(D), KF = med_f32_stride(D);
    if (bzero && blockIdx.x == 0)
        for (int e = threadIdx.x; e < NBK; e += blockDim.x) bzero[e] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (st_out) *st_out = st_init; // predicted bracket
        if (nmax_zero) *nmax_zero = 0;
    }
    __shared__ double mu[D];
    __shared__ double sP[4096];
    // the first row's X is loaded before the centre (its latency overlaps the
    // partials'), each later row's one iteration ahead
    const int64_t jstride = (int64_t)gridDim.x * blockDim.x;
    int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double xn[D], rs[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
        xn[k] = j < n ? X[j * D + k] : 0.0;
        rs[k] = 0.0;
    }
    center_mean<D>(pin, nin, n, sP, mu);
    unsigned long long bmax = 0;
    for (; j < np; j += jstride) {
        double v[KP];
        const bool live = j < n;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            v[k] = xn[k];
            rs[k] += xn[k]; // (zero past n)
        }
        const int64_t jn = j + jstride;
#pragma unroll
        for (int k = 0; k < D; ++k) xn[k] = jn < n ? X[jn * D + k] : 0.0;
#pragma unroll
        for (int k = 0; k < D; ++k) v[k] = live ? v[k] - mu[k] : 0.0;
#pragma unroll
        for (int k = D; k < KP; ++k) v[k] = 0.0;
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < D; ++k) s = fma(v[k], v[k], s); // (the zero pads add nothing)
        nrm[j] = s;
        float f[KF];
        if (xf) {
#pragma unroll
            for (int k = 0; k < KF; ++k)
                f[k] = k < D ? (float)v[k] : (k == D ? (live ? (float)(-0.5 * s) : -__builtin_inff()) : 0.0f);
        }
        if (nrm_in_slot) v[D] = -0.5 * s;
        double2 *o = reinterpret_cast<double2 *>(xc + j * KP);
#pragma unroll
        for (int q = 0; q < KP / 2; ++q) o[q] = make_double2(v[2 * q], v[2 * q + 1]);
        if (xf) {
            float4 *of = reinterpret_cast<float4 *>(xf + j * KF);
#pragma unroll
            for (int q = 0; q < KF / 4; ++q) of[q] = make_float4(f[4 * q], f[4 * q + 1], f[4 * q + 2], f[4 * q + 3]);
            if constexpr (D <= 8) {
                if (xs) { // the collect's split-bf16 operands [hi | lo] (zero past n)
                    float x8[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) x8[k] = k < D ? f[k] : 0.0f;
                    xs[2 * j] = mcol_split_bf16(x8, false);
                    xs[2 * j + 1] = mcol_split_bf16(x8, true);
                }
            }
            unsigned long long m = (unsigned long long)__double_as_longlong(s);
            for (int o2 = 32; o2 > 0; o2 >>= 1) {
                const unsigned long long t = __shfl_xor(m, o2);
                m = t > m ? t : m;
            }
            bmax = m > bmax ? m : bmax;
        }
    }
    // the block's column sums of X (pout): every thread's row sums to LDS
    // (sP is free again), then thread k < D adds column k's 256 in thread order
    if (pout) {
        __syncthreads(); // every block-mate is past its reads of sP
#pragma unroll
        for (int k = 0; k < D; ++k) sP[k * 256 + threadIdx.x] = rs[k];
    }
    if (xf) {
        __shared__ unsigned long long wmax[4];
        if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = bmax;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long m = 0;
            for (int w = 0; w < (int)(blockDim.x >> 6); ++w) m = wmax[w] > m ? wmax[w] : m;
            atomicMax(nmax_bits, m);
        }
    } else {
        __syncthreads();
    }
    if (pout) {
        // column k's 256 row sums: TC threads each add 256 / TC consecutive
        // ones, then a fixed shuffle tree (a column's threads are one aligned
        // lane group of a wave)
        constexpr int TC = D <= 4 ? 64 : D <= 8 ? 32 : 16, NV = 256 / TC;
        const int kc = threadIdx.x / TC, qc = threadIdx.x - kc * TC;
        double a = 0.0;
        if (kc < D) {
            const double *col = sP + kc * 256 + qc * NV;
#pragma unroll
            for (int t = 0; t < NV; ++t) a += col[t];
        }
#pragma unroll
        for (int h = TC / 2; h > 0; h >>= 1) a += __shfl_xor(a, h);
        if (kc < D && qc == 0) pout[(int64_t)blockIdx.x * D + kc] = a;
    }
}

// k_center for the tile path, KP = 32 / 64 (d > 16): the same values bit for
// bit (xc = X - mu, |xc|^2 as one fma chain over k ascending, the zero pads
// adding nothing), but the mean from the partials in one LDS sweep, the
// row's X loads unrolled and issued before the mean is formed (the generic
// loop, KP a run-time value, was a chain of dependent round trips: 77 us at
// N = 65536, d = 64), 16-byte record stores -- and, for SVGD_F32, the fp32
// copies the median passes read (xcf = fl(xc), nrmf = fl(|xc|^2), +inf in
// the padding rows: launch_cvt_nrm_f32) in the same pass, two launches fewer.
template <int KP>
__global__ __launch_bounds__(256) void k_center_t(const double *__restrict__ X, int64_t n, int d,
                                                  const double *__restrict__ partial, int nparts,
                                                  int64_t np, double *__restrict__ xc,
                                                  double *__restrict__ nrm, float *__restrict__ xcf,
                                                  float *__restrict__ nrmf, unsigned long long *bzero,
                                                  SelState *st_out, SelState st_init)
{
    if (bzero && blockIdx.x == 0)
        for (int e = threadIdx.x; e < NBK; e += blockDim.x) bzero[e] = 0;
    if (st_out && blockIdx.x == 0 && threadIdx.x == 0) *st_out = st_init;
    __shared__ double mu[KP];
    __shared__ double sP[4096];
    const int64_t jstride = (int64_t)gridDim.x * blockDim.x;
    int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // the first row's X loaded before the mean (its latency overlaps the
    // partials'; the grid usually gives each thread one row)
    double v[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) v[k] = (j < n && k < d) ? X[j * d + k] : 0.0;
    if (nparts * d <= 4096) {
        for (int e = threadIdx.x; e < nparts * d; e += blockDim.x) sP[e] = partial[e];
        __syncthreads();
        if (threadIdx.x < d) {
            double s = 0.0; // partials added in b order, as k_center
            int b = 0;
            for (; b + 8 <= nparts; b += 8) {
                double v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = sP[(b + u) * d + threadIdx.x];
#pragma unroll
                for (int u = 0; u < 8; ++u) s += v[u];
            }
            for (; b < nparts; ++b) s += sP[b * d + threadIdx.x];
            mu[threadIdx.x] = s / (double)n;
        }
    } else if (threadIdx.x < d) {
        const int k = threadIdx.x;
        double s = 0.0;
        for (int b0 = 0; b0 < nparts; b0 += 8) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = b0 + u < nparts ? partial[(b0 + u) * d + k] : 0.0;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (b0 + u < nparts) s += v[u];
        }
        mu[k] = s / (double)n;
    }
    __syncthreads();
    for (bool first = true; j < np; j += jstride, first = false) {
        const bool live = j < n;
        if (!first) {
#pragma unroll
            for (int k = 0; k < KP; ++k) v[k] = (live && k < d) ? X[j * d + k] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < KP; ++k) v[k] = (live && k < d) ? v[k] - mu[k] : 0.0;
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < KP; ++k) s = fma(v[k], v[k], s);
        nrm[j] = s;
        double2 *o = reinterpret_cast<double2 *>(xc + j * KP);
#pragma unroll
        for (int q = 0; q < KP / 2; ++q) o[q] = make_double2(v[2 * q], v[2 * q + 1]);
        if (xcf) {
            float4 *of = reinterpret_cast<float4 *>(xcf + j * KP);
#pragma unroll
            for (int q = 0; q < KP / 4; ++q)
                of[q] = make_float4((float)v[4 * q], (float)v[4 * q + 1], (float)v[4 * q + 2], (float)v[4 * q + 3]);
            nrmf[j] = live ? (float)s : __builtin_inff();
        }
    }
}

// V_j = [G_j - 2a xc_j, 1, 0...] (row stride 16*NCB), c_j = -a log2e |xc_j|^2.
__global__ void k_prep_v(const double *__restrict__ xc, const double *__restrict__ G,
                         const double *__restrict__ nrm, const double *__restrict__ a_ptr,
                         int64_t n, int64_t np, int d, int KP, int VW,
                         double *__restrict__ V, double *__restrict__ cvec)
{
    // one thread per element of V (coalesced stores; a thread per particle
    // wrote 16 NCB-strided doubles: 76 -> ~20 us at N = 65536, d = 64)
    const double a = *a_ptr;
    const int64_t tot = np * VW;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = e / VW;
        const int c = (int)(e - j * VW);
        double v = 0.0;
        if (j < n) {
            if (c < d) v = G[j * d + c] - 2.0 * a * xc[j * KP + c];
            else if (c == d) v = 1.0;
        }
        V[e] = v;
        if (c == 0) cvec[j] = j < n ? -a * LOG2E * nrm[j] : 0.0;
    }
}

// ------------------------------------------------------------------ phi --
//
// One workgroup = NW waves = 16 NW rows i (wave w: rows 16w..16w+15).  The
// workgroup sweeps all column tiles of 64 particles j staged through LDS.
// Per 16(j) x 16(i) sub-tile:
//   Gram   dot[j][i] = xc_j . xc_i     KP/4 MFMAs (A = X_J from LDS, B = X_I regs)
//   VALU   t = c_i + c_j + 2a log2e dot  ( = -a log2e |x_i - x_j|^2 )
//          P = 2^t                      (lane l: i = l&15, j = acc_row(l>>4, r))
//   MFMA   acc[i][c] += sum_j P[i][j] V[j][c]   (P is already the A-operand map)
// Epilogue: phi_i = (acc[i][0:d] + 2a xc_i acc[i][d]) / N (fp64).
// T = double (default) or float (SVGD_F32: Gram, exp and contraction on
// v_mfma_f32_16x16x4f32 / v_exp_f32 from fp32 copies xg, cvec, V).
//
// LDS layout (bank-conflict-free for the MFMA operand reads, whose lanes
// (lo, hi) touch rows lo / hi + 4r): X_J is j-major with row stride LDK, an
// odd multiple of 4 elements (the 16 lo rows x 4 hi columns of a Gram
// A-operand land in distinct banks; the fill is a straight 16-byte copy), and
// V_J rows are padded to VWP.  fp64 d = 64 thus needs 76 KB (was 124 KB with a
// k-major X_J and a separate epilogue buffer, 1 block of 4 waves per CU): the
// epilogue's per-wave accumulator tiles now reuse the staging buffers, in as
// many phases as needed, and an 8-wave block keeps 2 blocks = 4 waves/SIMD.
template <class T, int KP> struct PhiTile {
    static constexpr int LDK = ((KP / 4) & 1) ? KP : KP + 4;
};
template <class T, int VW> struct PhiVPad;
template <int VW> struct PhiVPad<double, VW> {
    static constexpr int VWP = ((VW / 16) & 1) ? VW : VW + 16;
};
template <int VW> struct PhiVPad<float, VW> {
    static constexpr int VWP = VW + 4;
};
template <class T, int KP, int NCB> struct PhiLds {
    static constexpr int VW = 16 * NCB, LDK = PhiTile<T, KP>::LDK, VWP = PhiVPad<T, VW>::VWP;
    static constexpr int XB = TB * LDK * (int)sizeof(T), VB = TB * VWP * (int)sizeof(T);
    static constexpr int MAIN = XB + VB + TB * (int)sizeof(T);
    static constexpr int ACCW = 16 * (VW + 1) * (int)sizeof(T); // one wave's epilogue tile
};

#ifndef SVGD_PHI_WPE
#define SVGD_PHI_WPE 1
#endif
// S1V (d = 16 NCB, fp64 d = 32/48/64): V holds no column of ones; the row
// sums s1_i = sum_j P_ij are added on the VALU (16 adds per tile and lane
// instead of a whole 16-column MFMA block: d = 64 runs 4 blocks, not 5), the
// padded columns j >= n masked through c_j = -huge (P = 0).
template <class T, int KP, int NCB, int NW, bool PRE, bool S1V>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(SVGD_PHI_WPE))) void k_phi(const T *__restrict__ xg, const T *__restrict__ cvec,
                                                 const T *__restrict__ V,
                                                 const double *__restrict__ a_ptr, int64_t row0,
                                                 int64_t nrows, int64_t ntiles_j, int64_t n, int d,
                                                 double inv_n, const double *__restrict__ wv,
                                                 const double *__restrict__ xc,
                                                 double *__restrict__ phi)
{
    typedef typename Acc4<T>::type A4;
    typedef PhiLds<T, KP, NCB> L;
    constexpr int VW = L::VW, LDK = L::LDK, VWP = L::VWP, NT = 64 * NW;
    constexpr int NWE = L::MAIN / L::ACCW < NW ? L::MAIN / L::ACCW : NW; // waves per epilogue phase
    static_assert(NWE >= 1, "phi epilogue tile exceeds the staging buffers");
    __shared__ __attribute__((aligned(16))) char smem[L::MAIN];
    T *sX = reinterpret_cast<T *>(smem);
    T *sV = reinterpret_cast<T *>(smem + L::XB);
    T *sC = reinterpret_cast<T *>(smem + L::XB + L::VB);

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int lo = lane & 15, hi = lane >> 4;
    const double a = *a_ptr;
    const T alpha = (T)(2.0 * a * LOG2E);

    const int64_t ibase = row0 + (int64_t)blockIdx.x * (16 * NW) + w * 16;
    // rows past the slice read its last row (valid memory; never stored)
    const int64_t il_ld = ibase + lo < row0 + nrows ? ibase + lo : row0 + nrows - 1;
    // B operand of the Gram MFMA: X_I^T, lane holds xg[i = lo][k = 4kk + hi]
    T bI[KP / 4];
#pragma unroll
    for (int kk = 0; kk < KP / 4; ++kk) bI[kk] = xg[il_ld * KP + 4 * kk + hi];
    const T ci = cvec[il_ld];

    A4 acc[NCB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) acc[cb] = A4{0, 0, 0, 0};
    T ps = (T)0; // S1V: this lane's share of s1_i (i = lo)
    const T CPAD = S1V ? (T)-1.0e300 : (T)0; // (fp32: -inf)

    // 16-byte pieces: X_J row jl holds KP/EP of them, V_J row VW/EP
    constexpr int EP = 16 / (int)sizeof(T);
    constexpr int NXP = TB * KP / EP, NVP = TB * VW / EP;
    constexpr int PX = (NXP + NT - 1) / NT, PV = (NVP + NT - 1) / NT;
    uint4 preX[PRE ? PX : 1], preV[PRE ? PV : 1];
    T preC = (T)0;
    auto put = [&](int e, uint4 vx, bool isv) {
        if (!isv) {
            const int jl = e / (KP / EP), q = e - jl * (KP / EP);
            *reinterpret_cast<uint4 *>(sX + jl * LDK + q * EP) = vx;
        } else {
            const int jl = e / (VW / EP), q = e - jl * (VW / EP);
            *reinterpret_cast<uint4 *>(sV + jl * VWP + q * EP) = vx;
        }
    };
    auto fetch = [&](int64_t j0) {
#pragma unroll
        for (int u = 0; u < PX; ++u) {
            const int e = tid + NT * u;
            if (NXP % NT == 0 || e < NXP) preX[u] = reinterpret_cast<const uint4 *>(xg + j0 * KP)[e];
        }
#pragma unroll
        for (int u = 0; u < PV; ++u) {
            const int e = tid + NT * u;
            if (NVP % NT == 0 || e < NVP) preV[u] = reinterpret_cast<const uint4 *>(V + j0 * VW)[e];
        }
        if (tid < TB) preC = cvec[j0 + tid];
    };
    if (PRE && ntiles_j > 0) fetch(0);
    for (int64_t jt = 0; jt < ntiles_j; ++jt) {
        __syncthreads();
        if constexpr (PRE) {
#pragma unroll
            for (int u = 0; u < PX; ++u) {
                const int e = tid + NT * u;
                if (NXP % NT == 0 || e < NXP) put(e, preX[u], false);
            }
#pragma unroll
            for (int u = 0; u < PV; ++u) {
                const int e = tid + NT * u;
                if (NVP % NT == 0 || e < NVP) put(e, preV[u], true);
            }
            if (tid < TB) sC[tid] = !S1V || jt * TB + tid < n ? preC : CPAD;
        } else {
            const int64_t j0 = jt * TB;
            for (int e = tid; e < NXP; e += NT) put(e, reinterpret_cast<const uint4 *>(xg + j0 * KP)[e], false);
            for (int e = tid; e < NVP; e += NT) put(e, reinterpret_cast<const uint4 *>(V + j0 * VW)[e], true);
            if (tid < TB) sC[tid] = !S1V || j0 + tid < n ? cvec[j0 + tid] : CPAD;
        }
        __syncthreads();
        if (PRE && jt + 1 < ntiles_j) fetch((jt + 1) * TB);

#pragma unroll
        for (int js = 0; js < 4; ++js) {
            A4 dot = {0, 0, 0, 0};
#pragma unroll
            for (int kk = 0; kk < KP / 4; ++kk)
                dot = mfma16(sX[(js * 16 + lo) * LDK + 4 * kk + hi], bI[kk], dot);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int jl = js * 16 + acc_row<T>(hi, r);
                const T p = exp2_nonpos(fma(alpha, dot[r], ci + sC[jl]));
                if (S1V) ps += p;
#pragma unroll
                for (int cb = 0; cb < NCB; ++cb)
                    acc[cb] = mfma16(p, sV[jl * VWP + cb * 16 + lo], acc[cb]);
            }
        }
    }

    // epilogue (fp64): acc lane map row i = acc_row(hi, q), col c = lo (+16cb);
    // waves w with w / NWE == ph use slot w % NWE of the staging buffers
    const double two_a = 2.0 * a;
    T *sAcc = reinterpret_cast<T *>(smem) + (w % NWE) * 16 * (VW + 1);
    if (S1V) { // the 4 lane groups' shares of row lo, in fixed order
        ps += __shfl_xor(ps, 16);
        ps += __shfl_xor(ps, 32);
    }
    const int s1c = S1V ? VW : d;
#pragma unroll 1
    for (int ph = 0; ph < (NW + NWE - 1) / NWE; ++ph) {
        __syncthreads();
        if (w / NWE == ph) {
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
                for (int q = 0; q < 4; ++q) sAcc[acc_row<T>(hi, q) * (VW + 1) + cb * 16 + lo] = acc[cb][q];
            if (S1V && hi == 0) sAcc[lo * (VW + 1) + VW] = ps;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (int e = lane; e < 16 * d; e += 64) {
                const int il = e / d, c = e - il * d;
                const int64_t i = ibase + il;
                if (i - row0 < nrows) {
                    const double s1 = (double)sAcc[il * (VW + 1) + s1c];
                    const double wgt = wv ? wv[i * d + c] : two_a * xc[i * KP + c];
                    phi[(i - row0) * d + c] = inv_n * ((double)sAcc[il * (VW + 1) + c] + wgt * s1);
                }
            }
        }
    }
}

// ----------------------------------------------------------- optimizers --
// Elementwise, bit-exact with the reference expressions (no FMA contraction).

// bak (optional, the speculative step): bak[0..cnt) = X_t, bak[cnt..2cnt) =
// m_t, bak[2cnt..3cnt) = v_t of these elements, written in the same pass.
// An element's optimizer state, loaded ahead of the phi value it needs
// (k_phi_reduce issues these loads before its partial sums)
struct OptIn {
    double m, v, x;
};
__device__ __forceinline__ OptIn opt_load(const OptArgs &o, int64_t e)
{
    return OptIn{o.kind == 0 ? o.m[e] : 0.0, o.v[e], o.X[e]};
}
__device__ __forceinline__ double opt_apply(const OptArgs &o, int64_t e, double ge, const OptIn &in)
{
#pragma clang fp contract(off)
    if (o.bak) {
        o.bak[e] = in.x;
        o.bak[o.cnt + e] = o.kind == 0 ? in.m : o.m[e];
        o.bak[2 * o.cnt + e] = in.v;
    }
    double delta;
    if (o.kind == 0) { // Adam.hpp:75-83
        const double me = o.b1 * in.m + (1 - o.b1) * ge;
        const double ve = o.b2 * in.v + (1 - o.b2) * (ge * ge);
        o.m[e] = me;
        o.v[e] = ve;
        delta = (o.lr * (1.0 / (o.eps + sqrt(ve / o.c2)))) * (me / o.c1);
    } else if (o.kind == 1) { // AdaGrad.hpp:60-65
        const double ve = in.v + ge * ge;
        o.v[e] = ve;
        delta = (o.lr * (1.0 / (o.eps + sqrt(ve)))) * ge;
    } else { // RMSProp.hpp:69-74 (beta passed as b1)
        const double ve = o.b1 * in.v + (1 - o.b1) * (ge * ge);
        o.v[e] = ve;
        delta = (o.lr * (1.0 / (o.eps + sqrt(ve)))) * ge;
    }
    double x = in.x + delta; // SVGD.hpp:393
    if (o.lower) {           // SVGD.hpp:396-399: min(upper) then max(lower)
        const int k = (int)(e % o.d);
        x = x < o.upper[k] ? x : o.upper[k];
        x = x > o.lower[k] ? x : o.lower[k];
    }
    o.X[e] = x;
    if (o.xh) o.xh[e] = x; // the host gradient's copy of X_{t+1} (no D2H copy)
    return x;
}
__device__ __forceinline__ double opt_elem(const OptArgs &o, int64_t e, double ge)
{
    return opt_apply(o, e, ge, opt_load(o, e));
}

__global__ void k_opt_update(OptArgs o, const double *__restrict__ g)
{
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < o.cnt;
         e += (int64_t)gridDim.x * blockDim.x)
        opt_elem(o, e, g[e]);
}

// --------------------------------------------------------------- median --
// (keys, key-range buckets, the tile plan and the pass sinks: svgd_device.h)

__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// next representable value towards +inf of a finite non-negative float/double
__device__ __forceinline__ float nextafter_up(float x)
{
    return __int_as_float(__float_as_int(x) + 1);
}
__device__ __forceinline__ double nextafter_up(double x)
{
    return __longlong_as_double(__double_as_longlong(x) + 1);
}

template <class T, int KP, int MODE>
__global__ __launch_bounds__(256) void k_pair_tiles(const T *__restrict__ xc,
                                                   const T *__restrict__ nrm, int64_t n,
                                                   int64_t nb, int64_t t0, int64_t t1,
                                                   SinkCollect sc, SinkHist sh, SinkDebug sd,
                                                   const uint32_t *__restrict__ xk)
{
    typedef typename Acc4<T>::type A4;
    // F32 at KP 32 / 64: the bf16 part-product keys from the key parts xk
    // (svgd_device.h), no X tiles in LDS
    constexpr bool B3K = sizeof(T) == 4 && kb3_keys(KP);
    // fp64: the X tiles j-major with row stride LDK (an odd multiple of 4
    // doubles: the MFMA operand reads of 16 rows x 4 columns hit distinct
    // banks, the fill is a straight 16-byte copy) -- 70 KB instead of 80 KB
    // of tiles, so two work-groups fit a CU (round 3: one, 1 wave/SIMD);
    // fp32 keeps the k-major tiles (its kslot order would conflict j-major)
    constexpr bool JM = sizeof(T) == 8 && (KP / 4) % 2 == 0;
    constexpr int LDK = PhiTile<T, KP>::LDK;
    constexpr int XT = B3K ? 4 : JM ? TB * LDK : KP * LDP;
    __shared__ __attribute__((aligned(16))) T sXI[XT];
    __shared__ __attribute__((aligned(16))) T sXJ[XT];
    __shared__ T sNI[TB], sNJ[TB];
    __shared__ uint32_t sHist[(MODE == 1) ? 2 * RADIX : 1];
    __shared__ uint32_t sCnt;
    __shared__ unsigned long long sBelow[4];
    __shared__ uint32_t sBk[(MODE == 0) ? NBK : 1];

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int lo = lane & 15, hi = lane >> 4;

    const int64_t ntiles = t1 - t0;
    const int64_t tb = t0 + ntiles * blockIdx.x / gridDim.x;
    const int64_t te = t0 + ntiles * (blockIdx.x + 1) / gridDim.x;

    // MODE 1 (histogram) selection state
    int nsel = 0, shift = 0;
    uint64_t pfx[2] = {0, 0};
    int hsh = 63;
    if (MODE == 1) {
        nsel = sh.st->nsel;
        shift = sh.st->shift;
        hsh = shift + sh.st->width;
        pfx[0] = sh.st->prefix[0];
        pfx[1] = sh.st->prefix[1];
        for (int e = tid; e < 2 * RADIX; e += 256) sHist[e] = 0;
    }
    uint64_t lo_key = 0, hi_key = 0;
    double binv = 0.0;
    // MODE 0 classifies s in the kernel's precision: for non-negative s,
    // key_of(s) < lo_key <=> s < loT with loT the smallest T >= the double of
    // lo_key (keys of non-negative doubles order like the doubles; fp32 keys
    // widen exactly), likewise hi; the key itself is formed in the band only
    T loT = (T)0, hiT = (T)0;
    if (MODE == 0) {
        lo_key = sc.st->lo_key;
        hi_key = sc.st->hi_key;
        binv = sc.st->binv;
        const double lo_d = __longlong_as_double((long long)lo_key);
        const double hi_d = hi_key >= 0x7ff0000000000000ull ? __builtin_inf()
                                                            : __longlong_as_double((long long)hi_key);
        loT = (T)lo_d;
        if ((double)loT < lo_d) loT = nextafter_up(loT);
        hiT = (T)hi_d;
        if ((double)hiT < hi_d) hiT = nextafter_up(hiT);
        if (tid == 0) sCnt = 0;
        if (sc.bpart)
            for (int e = tid; e < NBK; e += 256) sBk[e] = 0;
        __syncthreads();
    }
    uint32_t below = 0;

    auto coords = [&](int64_t t, int64_t *I, int64_t *J) {
        if (MODE == 3) {
            // sample tile t: a random pair of distinct full 64-particle blocks
            const uint64_t h = mix64((uint64_t)t * 2 + 1);
            const int64_t nbf = sd.n / TB;
            *I = (int64_t)(h % (uint64_t)nbf);
            *J = (*I + 1 + (int64_t)((h >> 32) % (uint64_t)(nbf - 1))) % nbf;
        } else {
            tile_coords(nb, t, I, J);
        }
    };
    // the next tile's column block is loaded into registers while the current
    // tile is computed, then stored to LDS between the two barriers
    constexpr int PU = TB * KP / 256;
    constexpr int EP = 16 / (int)sizeof(T), PQ = JM ? PU / EP : 1; // 16-byte pieces
    static_assert(!JM || PU % EP == 0, "tile pieces");
    T preX[JM ? 1 : PU];
    uint4 preQ[PQ];
    T preN = (T)0;
    auto fetch = [&](int64_t Jn) {
        if constexpr (B3K) {
        } else if constexpr (JM) {
#pragma unroll
            for (int u = 0; u < PQ; ++u)
                preQ[u] = reinterpret_cast<const uint4 *>(xc + Jn * TB * KP)[tid + 256 * u];
        } else {
#pragma unroll
            for (int u = 0; u < PU; ++u) {
                const int e = tid + 256 * u, jl = e / KP, k = e - jl * KP;
                preX[u] = xc[(Jn * TB + jl) * KP + k];
            }
        }
        if (tid < TB) preN = nrm[Jn * TB + tid];
    };
    // piece e of a 64-particle block (row jl = e / (KP/EP)) into a j-major tile
    auto put = [&](T *dst, int e, uint4 v) {
        const int jl = e / (KP / EP), q = e - jl * (KP / EP);
        *reinterpret_cast<uint4 *>(dst + jl * LDK + q * EP) = v;
    };
    int64_t curI = -1, I = 0, J = 0;
    if (tb < te) {
        coords(tb, &I, &J);
        fetch(J);
    }
    for (int64_t t = tb; t < te; ++t) {
        __syncthreads();
        if (I != curI) {
            if constexpr (B3K) {
            } else if constexpr (JM) {
                for (int e = tid; e < TB * KP / EP; e += 256)
                    put(sXI, e, reinterpret_cast<const uint4 *>(xc + I * TB * KP)[e]);
            } else {
                for (int e = tid; e < TB * KP; e += 256) {
                    const int il = e / KP, k = e - il * KP;
                    sXI[k * LDP + il] = xc[(I * TB + il) * KP + k];
                }
            }
            if (tid < TB) sNI[tid] = nrm[I * TB + tid];
        }
        if constexpr (B3K) {
        } else if constexpr (JM) {
#pragma unroll
            for (int u = 0; u < PQ; ++u) put(sXJ, tid + 256 * u, preQ[u]);
        } else {
#pragma unroll
            for (int u = 0; u < PU; ++u) {
                const int e = tid + 256 * u, jl = e / KP, k = e - jl * KP;
                sXJ[k * LDP + jl] = preX[u];
            }
        }
        if (tid < TB) sNJ[tid] = preN;
        __syncthreads();
        curI = I;
        const int64_t Ic = I, Jc = J;
        if (t + 1 < te) {
            coords(t + 1, &I, &J);
            fetch(J);
        }

        const bool full = Ic != Jc && (Ic + 1) * TB <= n && (Jc + 1) * TB <= n;
        T bI[B3K ? 1 : KP / 4];
        if constexpr (!B3K) {
#pragma unroll
            for (int kk = 0; kk < KP / 4; ++kk)
                bI[kk] = JM ? sXI[(w * 16 + lo) * LDK + kslot<T, KP>(kk, hi)]
                            : sXI[kslot<T, KP>(kk, hi) * LDP + w * 16 + lo];
        }
        // B3K, a wrapped tile (J < I): the rows take the A role (larger
        // indices), so the lane map is transposed: row 4 hi + r, column lo
        const bool swp = B3K && Jc < Ic;

#pragma unroll
        for (int js = 0; js < 4; ++js) {
            A4 dot = {0, 0, 0, 0};
            if constexpr (B3K) {
                const uint32_t *pr = xk + (Ic * 4 + w) * kb3_block_words(KP) + lane * 4;
                const uint32_t *pc = xk + (Jc * 4 + js) * kb3_block_words(KP) + lane * 4;
                dot = kb3_dot<KP>(swp ? pr : pc, swp ? pc : pr);
            } else {
#pragma unroll
                for (int kk = 0; kk < KP / 4; ++kk)
                    dot = mfma16(JM ? sXJ[(js * 16 + lo) * LDK + kslot<T, KP>(kk, hi)]
                                    : sXJ[kslot<T, KP>(kk, hi) * LDP + js * 16 + lo],
                                 bI[kk], dot);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int jl = swp ? js * 16 + lo : js * 16 + acc_row<T>(hi, r);
                const int il = swp ? w * 16 + acc_row<T>(hi, r) : w * 16 + lo;
                const int64_t i = Ic * TB + il, j = Jc * TB + jl;
                const T ni = sNI[il];
                if constexpr (MODE == 0) {
                    // off-diagonal tiles of two full blocks (all but a few):
                    // every pair is valid
                    const bool valid = full || ((i < n) && (j < n) && (Ic != Jc || il < jl));
                    const T sv = fmax(fma((T)-2, dot[r], ni + sNJ[jl]), (T)0);
                    const bool isb = sv < loT;
                    const bool in = valid && !isb && sv < hiT;
                    below += (valid && isb) ? 1u : 0u;
                    const unsigned long long mask = __ballot(in);
                    if (mask) {
                        uint32_t base = 0;
                        if (lane == 0) base = atomicAdd(&sCnt, (uint32_t)__popcll(mask));
                        base = __shfl(base, 0);
                        if (in) {
                            // key of the distance in the kernel's precision
                            const uint64_t key = key_of((double)sv);
                            const int64_t pos =
                                base + __popcll(mask & ((1ull << lane) - 1ull));
                            if (pos < sc.cap) sc.region[blockIdx.x * sc.cap + pos] = key;
                            if (sc.bpart) atomicAdd(&sBk[kbucket(key, lo_key, binv)], 1u);
                        }
                    }
                    continue;
                }
                const bool valid = (i < n) && (j < n) && (Ic != Jc || il < jl);
                // key of the distance in the kernel's precision (fp32 keys widen exactly)
                const double s = (double)fmax(fma((T)-2, dot[r], ni + sNJ[jl]), (T)0);
                const uint64_t key = key_of(s);
                if (MODE == 1) {
                    if (valid) {
                        for (int s2 = 0; s2 < nsel; ++s2) {
                            const bool match = hsh >= 64 || (key >> hsh) == (pfx[s2] >> hsh);
                            if (match)
                                atomicAdd(&sHist[s2 * RADIX + ((key >> shift) & (RADIX - 1))], 1u);
                        }
                    }
                } else if (MODE == 3) {
                    sd.keys[t * (TB * TB) + il * TB + jl] = key;
                } else {
                    if (valid) {
                        const int64_t a = i < j ? i : j, b = i < j ? j : i;
                        const int64_t idx = a * (2 * sd.n - a - 1) / 2 + (b - a - 1);
                        sd.out[idx] = s;
                    }
                }
            }
        }
    }

    if (MODE == 0) {
        // block reduce `below`
        unsigned long long bl = below;
        for (int o = 32; o > 0; o >>= 1) bl += __shfl_down(bl, o);
        if (lane == 0) sBelow[w] = bl;
        __syncthreads();
        if (tid == 0) {
            sc.below_out[blockIdx.x] = sBelow[0] + sBelow[1] + sBelow[2] + sBelow[3];
            sc.count_out[blockIdx.x] = sCnt;
        }
        if (sc.bpart)
            for (int e = tid; e < NBK; e += 256) sc.bpart[(int64_t)blockIdx.x * NBK + e] = sBk[e];
    } else if (MODE == 1) {
        __syncthreads();
        for (int e = tid; e < 2 * RADIX; e += 256)
            if (sHist[e]) atomicAdd(&sh.ghist[e], (unsigned long long)sHist[e]);
    }
}

// Sampled keys: pair (i, j != i) from a splitmix hash of the sample index;
// region b holds keys [b*per, (b+1)*per).

// st_out (optional): the bracket passes' initial select state, written here
// so it needs no launch of its own (kernel arguments are captured at launch).
__global__ void k_sample_keys(const double *__restrict__ xc, const double *__restrict__ nrm,
                              int64_t n, int d, int KP, int64_t g0, int64_t S,
                              uint64_t *__restrict__ keys, SelState init, SelState *st_out)
{
    if (st_out && blockIdx.x == 0 && threadIdx.x == 0) *st_out = init;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < S;
         g += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t h = mix64((uint64_t)(g0 + g) * 2 + 1);
        const int64_t i = (int64_t)(h % (uint64_t)n);
        const int64_t j = (i + 1 + (int64_t)((h >> 32) % (uint64_t)(n - 1))) % n;
        double dot = 0.0;
        for (int k = 0; k < d; ++k) dot = fma(xc[i * KP + k], xc[j * KP + k], dot);
        keys[g] = key_of(fmax(fma(-2.0, dot, nrm[i] + nrm[j]), 0.0));
    }
}

// Sampled keys from the fp32 records (d <= 16): one random upper-triangle
// pair per thread, each record read with KF/4 16-byte loads.  The keys only
// place the bracket, whose exactness the collect pass checks.
__device__ __forceinline__ int64_t mulhi_index(uint32_t r, int64_t n)
{
    return (int64_t)(((uint64_t)r * (uint64_t)n) >> 32);
}

template <int D>
__global__ __launch_bounds__(256) void k_sample_keys_f32(const float *__restrict__ xf, int64_t n,
                                                         int64_t g0, int64_t S,
                                                         uint64_t *__restrict__ keys, SelState init,
                                                         SelState *st_out)
{
    if (st_out && blockIdx.x == 0 && threadIdx.x == 0) *st_out = init;
    constexpr int KF = med_f32_stride(D);
    // SU samples per thread with their record loads in flight together
    constexpr int SU = 1; // (4 in flight measured slower: occupancy, L2-rate bound)
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    // (g: this rank's sample slot; g0 + g: the index in the one global sequence)
    for (int64_t gb = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; gb < S; gb += stride * SU) {
        float4 ra[SU][KF / 4], rb[SU][KF / 4];
#pragma unroll
        for (int u = 0; u < SU; ++u) {
            const int64_t g = gb + u * stride;
            const uint64_t h = mix64((uint64_t)(g0 + (g < S ? g : 0)) * 2 + 1);
            const int64_t i = mulhi_index((uint32_t)(h >> 32), n);
            int64_t j = i + 1 + mulhi_index((uint32_t)h, n - 1);
            if (j >= n) j -= n;
            const float4 *ri = reinterpret_cast<const float4 *>(xf + i * KF);
            const float4 *rj = reinterpret_cast<const float4 *>(xf + j * KF);
#pragma unroll
            for (int q = 0; q < KF / 4; ++q) {
                ra[u][q] = ri[q];
                rb[u][q] = rj[q];
            }
        }
#pragma unroll
        for (int u = 0; u < SU; ++u) {
            const int64_t g = gb + u * stride;
            if (g >= S) break;
            const float *a = reinterpret_cast<const float *>(ra[u]);
            const float *b = reinterpret_cast<const float *>(rb[u]);
            float e = a[D] + b[D]; // -(n_i + n_j) / 2
#pragma unroll
            for (int k = 0; k < D; ++k) e = fmaf(a[k], b[k], e);
            keys[g] = key_of(fmax(-2.0 * (double)e, 0.0));
        }
    }
}

// Histogram of keys in `nreg` regions (region r: keys[r*cap .. r*cap+cnt_r)),
// cnt_r = counts ? min(counts[r], cap) : cap, for the current digit of each
// active selection (keys whose resolved high bits match its prefix).  Block b
// of HIST_BLOCKS (or fewer) takes regions b, b + G, ... (nreg >= G) or one of
// G / nreg slices of a region and adds its LDS histogram's non-zero bins into
// ghist (64-bit integer atomics, order-free; the keys of one digit crowd into
// few bins, so a block flushes few) -- one launch per pass, no partials sum.
// ghist is zero on entry (k_select_scan clears it after each pass).
constexpr int HIST_BLOCKS = 256;
__global__ __launch_bounds__(256) void k_hist_regions(const uint64_t *__restrict__ keys,
                                                     const uint32_t *__restrict__ counts,
                                                     int64_t nreg, int64_t cap,
                                                     const SelState *__restrict__ st,
                                                     unsigned long long *__restrict__ ghist)
{
    __shared__ uint32_t sHist[2 * RADIX];
    for (int e = threadIdx.x; e < 2 * RADIX; e += 256) sHist[e] = 0;
    __syncthreads();
    const int nsel = st->nsel, shift = st->shift, hsh = shift + st->width;
    const uint64_t p0 = st->prefix[0], p1 = st->prefix[1];
    const int64_t G = gridDim.x;
    const int64_t parts = nreg >= G ? 1 : G / nreg;
    const int64_t rstep = nreg >= G ? G : nreg;
    const int64_t part = nreg >= G ? 0 : blockIdx.x % parts;
    for (int64_t r = nreg >= G ? blockIdx.x : blockIdx.x / parts; r < nreg; r += rstep) {
        if (nreg < G && (int64_t)blockIdx.x >= parts * nreg) break;
        int64_t cnt = counts ? (int64_t)counts[r] : cap;
        if (cnt > cap) cnt = cap;
        const uint64_t *kr = keys + r * cap;
        // HU independent loads in flight per thread (the loop is latency bound)
        constexpr int HU = 8;
        for (int64_t e0 = part * 256 * HU + threadIdx.x; e0 < cnt; e0 += parts * 256 * HU) {
            uint64_t kk[HU];
#pragma unroll
            for (int u = 0; u < HU; ++u) {
                const int64_t e = e0 + u * 256;
                kk[u] = e < cnt ? kr[e] : 0;
            }
#pragma unroll
            for (int u = 0; u < HU; ++u) {
                if (e0 + u * 256 >= cnt) break;
                const uint64_t key = kk[u];
                const uint32_t dg = (uint32_t)((key >> shift) & (RADIX - 1));
                if (hsh >= 64 || (key >> hsh) == (p0 >> hsh)) atomicAdd(&sHist[dg], 1u);
                if (nsel > 1 && (hsh >= 64 || (key >> hsh) == (p1 >> hsh)))
                    atomicAdd(&sHist[RADIX + dg], 1u);
            }
        }
        if (nreg < G) break;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 2 * RADIX; e += 256)
        if (sHist[e]) atomicAdd(&ghist[e], (unsigned long long)sHist[e]);
}

// Keys of the regions whose resolved high bits (>= shift + width after the
// last k_select_scan) match either selection's prefix -> cbuf, count in
// *ccount (order of the compacted keys is irrelevant to the selection).
__global__ __launch_bounds__(256) void k_compact(const uint64_t *__restrict__ keys,
                                                const uint32_t *__restrict__ counts, int64_t nreg,
                                                int64_t cap, const SelState *__restrict__ st,
                                                uint64_t *__restrict__ cbuf,
                                                unsigned long long *__restrict__ ccount)
{
    __shared__ int sCnt[4];
    __shared__ unsigned long long sBase;
    const int nsel = st->nsel, hsh = st->shift + st->width;
    const uint64_t p0 = st->prefix[0], p1 = st->prefix[1];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int64_t r = blockIdx.x; r < nreg; r += gridDim.x) {
        int64_t cnt = counts ? (int64_t)counts[r] : cap;
        if (cnt > cap) cnt = cap;
        const uint64_t *kr = keys + r * cap;
        constexpr int CU = 8; // loads in flight per thread
        for (int64_t b = 0; b < cnt; b += 256 * CU) {
            uint64_t kk[CU];
            unsigned long long bal[CU];
            int wtot = 0;
#pragma unroll
            for (int u = 0; u < CU; ++u) {
                const int64_t e = b + u * 256 + threadIdx.x;
                kk[u] = e < cnt ? kr[e] : 0;
            }
#pragma unroll
            for (int u = 0; u < CU; ++u) {
                const int64_t e = b + u * 256 + threadIdx.x;
                const uint64_t key = kk[u];
                const bool m = e < cnt && (hsh >= 64 || (key >> hsh) == (p0 >> hsh) ||
                                           (nsel > 1 && (key >> hsh) == (p1 >> hsh)));
                bal[u] = __ballot(m);
                wtot += __popcll(bal[u]);
            }
            // one global atomic per block and chunk (a shared counter hit by
            // every wave with a match serialises at the L2)
            if (lane == 0) sCnt[w] = wtot;
            __syncthreads();
            if (threadIdx.x == 0) {
                const int tot = sCnt[0] + sCnt[1] + sCnt[2] + sCnt[3];
                sBase = tot ? atomicAdd(ccount, (unsigned long long)tot) : 0ull;
            }
            __syncthreads();
            unsigned long long base = sBase;
            for (int v = 0; v < w; ++v) base += sCnt[v];
#pragma unroll
            for (int u = 0; u < CU; ++u) {
                if ((bal[u] >> lane) & 1ull) cbuf[base + __popcll(bal[u] & ((1ull << lane) - 1ull))] = kk[u];
                base += __popcll(bal[u]);
            }
            __syncthreads(); // sCnt / sBase reused by the next chunk
        }
    }
}

// The remaining digits of the selection over the compacted keys, in one
// work-group (single rank only): per digit an LDS histogram of the matching
// keys and the same scan as k_select_scan.  Leaves st as the passes would.
__global__ __launch_bounds__(1024) void k_select_tail(SelState *st, const uint64_t *__restrict__ cbuf,
                                                     const unsigned long long *__restrict__ ccount,
                                                     int passes)
{
    __shared__ uint32_t sHist[2 * RADIX];
    __shared__ unsigned long long sPart[1024];
    __shared__ int sDigit;
    __shared__ unsigned long long sBelowD;
    const int tid = threadIdx.x;
    const int64_t cnt = (int64_t)*ccount;
    const int nsel = st->nsel;
    for (int p = 0; p < passes; ++p) {
        const int shift = st->shift, hsh = shift + st->width;
        const uint64_t p0 = st->prefix[0], p1 = st->prefix[1];
        for (int e = tid; e < 2 * RADIX; e += 1024) sHist[e] = 0;
        __syncthreads();
        for (int64_t e = tid; e < cnt; e += 1024) {
            const uint64_t key = cbuf[e];
            const uint32_t dg = (uint32_t)((key >> shift) & (RADIX - 1));
            if (hsh >= 64 || (key >> hsh) == (p0 >> hsh)) atomicAdd(&sHist[dg], 1u);
            if (nsel > 1 && (hsh >= 64 || (key >> hsh) == (p1 >> hsh)))
                atomicAdd(&sHist[RADIX + dg], 1u);
        }
        __syncthreads();
        constexpr int PER = RADIX / 1024;
        for (int s = 0; s < nsel; ++s) {
            const uint32_t *h = sHist + s * RADIX;
            unsigned long long loc = 0;
            for (int q = 0; q < PER; ++q) loc += h[tid * PER + q];
            sPart[tid] = loc;
            if (tid == 0) sDigit = -1;
            __syncthreads();
            for (int o = 1; o < 1024; o <<= 1) {
                const unsigned long long v = tid >= o ? sPart[tid - o] : 0ull;
                __syncthreads();
                sPart[tid] += v;
                __syncthreads();
            }
            const unsigned long long rank = st->rank[s];
            const unsigned long long excl = tid ? sPart[tid - 1] : 0ull;
            if (rank >= excl && rank < sPart[tid]) {
                unsigned long long c = excl;
                for (int q = 0; q < PER; ++q) {
                    const unsigned long long hv = h[tid * PER + q];
                    if (rank < c + hv) {
                        sDigit = tid * PER + q;
                        sBelowD = c;
                        break;
                    }
                    c += hv;
                }
            }
            __syncthreads();
            if (tid == 0) {
                if (sDigit < 0) {
                    st->error = 1;
                } else {
                    st->prefix[s] |= (uint64_t)sDigit << shift;
                    st->rank[s] = rank - sBelowD;
                }
            }
            __syncthreads();
        }
        if (tid == 0) {
            st->pass += 1;
            const int nshift = shift - RADIX_BITS;
            st->shift = nshift >= 0 ? nshift : 0;
            st->width = nshift >= 0 ? RADIX_BITS : shift;
        }
        __syncthreads();
    }
}

// ------------------------------------------------ bucket select path --
// Device-side bucket plan (the speculative step: no host round trip between
// the collect pass and the selection).  From the all-reduced counts: the
// order statistics are in the bracket (no overflowed region, r0 >= below,
// r1 < below + candidates), their buckets (svgd_plan_bucket_select's scan,
// here 256 threads x 8 buckets + a block scan) and the selected buckets'
// total <= capr.  Then the select state for k_compact_buckets /
// k_select_small, this rank's segment counter zeroed, *status = 0; otherwise
// *status = 1 (bracket miss), 2 (overflowed region) or 3 (selected buckets
// above capr) and the selection kernels do nothing -- the host redoes the step
// on its synchronous path.
// The status also goes to host_status (pinned host memory, read after the
// launch's completion event).
// The bucket plan of the speculative step, computed by one 256-thread block
// from the all-reduced counts: the buckets holding the order statistics and
// their ranks inside them, or status 1 (bracket miss), 2 (overflowed region),
// 3 (selected buckets above capr).  Block-uniform results.
struct PlanOut {
    int status, b0, b1, ns;
    unsigned long long in0, in1, tot;
};
__device__ PlanOut plan_block(const unsigned long long *__restrict__ cnt, int nsel, uint64_t r0,
                              uint64_t r1, int64_t capr, int sim = 0)
{
    __shared__ unsigned long long sPart[256];
    __shared__ int sB[2];
    __shared__ unsigned long long sIn[2];
    const int tid = threadIdx.x;
    PlanOut o{0, -1, -1, 1, 0, 0, 0};
    const unsigned long long below = cnt[0], cand = cnt[1], ovf = cnt[2];
    if (sim) { // measurement mode (PlanArgs::sim)
        const uint64_t dr = r1 - r0;
        r0 = below + cand / 2;
        r1 = r0 + dr;
    }
    if (ovf || r0 < below || r1 >= below + cand) {
        o.status = ovf ? 2 : 1;
        return o;
    }
    const unsigned long long q[2] = {r0 - below, r1 - below};
    const int ns = (nsel > 1 && q[1] != q[0]) ? 2 : 1;
    constexpr int PER = NBK / 256;
    unsigned long long loc = 0;
    for (int u = 0; u < PER; ++u) loc += cnt[3 + tid * PER + u];
    sPart[tid] = loc;
    if (tid < 2) sB[tid] = -1;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        const unsigned long long v = tid >= off ? sPart[tid - off] : 0ull;
        __syncthreads();
        sPart[tid] += v;
        __syncthreads();
    }
    const unsigned long long excl = tid ? sPart[tid - 1] : 0ull;
    for (int s = 0; s < ns; ++s)
        if (q[s] >= excl && q[s] < sPart[tid]) {
            unsigned long long c = excl;
            for (int u = 0; u < PER; ++u) {
                const unsigned long long h = cnt[3 + tid * PER + u];
                if (q[s] < c + h) {
                    sB[s] = tid * PER + u;
                    sIn[s] = q[s] - c;
                    break;
                }
                c += h;
            }
        }
    __syncthreads();
    if (sB[0] < 0 || (ns > 1 && sB[1] < 0)) {
        o.status = 1;
        return o;
    }
    o.ns = ns;
    o.b0 = sB[0];
    o.b1 = ns > 1 ? sB[1] : sB[0];
    o.in0 = sIn[0];
    o.in1 = ns > 1 ? sIn[1] : sIn[0];
    const unsigned long long tot = cnt[3 + o.b0] + (o.b1 != o.b0 ? cnt[3 + o.b1] : 0ull);
    o.tot = tot;
    if (tot > (unsigned long long)capr) o.status = 3;
    return o;
}

// The plan's select state and status (one thread); seg[0] (this rank's
// compaction counter) is zeroed by k_counts_reduce.
__device__ void plan_publish(const PlanOut &o, SelState *st, int nsel, int *status_d, int *status_h)
{
    if (o.status == 0) {
        st->nsel = nsel;
        st->rank[0] = o.in0;
        st->rank[1] = nsel > 1 ? o.in1 : o.in0;
        st->bsel[0] = o.b0;
        st->bsel[1] = o.b1;
        st->prefix[0] = st->prefix[1] = 0;
        st->error = 0;
    }
    *status_d = o.status;
    if (status_h) *status_h = o.status;
}

__global__ __launch_bounds__(256) void k_plan_select(const unsigned long long *__restrict__ cnt,
                                                    SelState *st, int nsel, uint64_t r0,
                                                    uint64_t r1, int64_t capr, uint64_t *seg,
                                                    int *status_arg, int *host_status)
{
    const PlanOut o = plan_block(cnt, nsel, r0, r1, capr);
    if (threadIdx.x != 0) return;
    if (o.status == 0) seg[0] = 0;
    plan_publish(o, st, nsel, status_arg, host_status);
}

// Whole select state / scale from kernel arguments (captured at launch, so the
// host never rewrites a staging buffer that an earlier queued copy still reads)
__global__ void k_set_state(SelState s, SelState *st) { *st = s; }
__global__ void k_set_scal(double a, double med, double *scal)
{
    scal[0] = a;
    scal[1] = med;
}

__global__ void k_set_sel(SelState *st, int nsel, uint64_t r0, uint64_t r1, int b0, int b1,
                          uint64_t *seg)
{
    seg[0] = 0; // compaction counter of this rank's segment
    st->nsel = nsel;
    st->rank[0] = r0;
    st->rank[1] = r1;
    st->bsel[0] = b0;
    st->bsel[1] = b1;
    st->prefix[0] = st->prefix[1] = 0;
    st->error = 0;
}

// Keys of the regions in the selected bucket(s) -> seg = [count, keys].  A
// block gathers its regions' matches in LDS and reserves output space with
// one global atomic per flush (a counter that every block hits per region
// serialises at the L2).  Positions past seg_cap are dropped: the host only
// takes this path when the selected buckets hold <= seg_cap keys in total.
constexpr int CB_LDS = 4096; // keys buffered per block between flushes
__global__ __launch_bounds__(256) void k_compact_buckets(const uint64_t *__restrict__ keys,
                                                        const uint32_t *__restrict__ counts,
                                                        int64_t nreg, int64_t cap,
                                                        SelState *__restrict__ st,
                                                        uint64_t *__restrict__ seg, int64_t seg_cap,
                                                        const int *__restrict__ status, PlanArgs pa)
{
    int nsel, b0, b1;
    if (pa.cnt) {
        // speculative step: every block derives the bucket plan from the
        // all-reduced counts itself (no plan launch); block 0 publishes it
        const PlanOut o = plan_block(pa.cnt, pa.nsel, pa.r0, pa.r1, pa.capr, pa.sim);
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (pa.trk) { // this step's bracket and counts for the host's bracket tracking
                pa.trk[0] = st->lo_key;
                pa.trk[1] = st->hi_key;
                pa.trk[2] = pa.cnt[0];
                pa.trk[3] = pa.cnt[1];
                pa.trk[7] = o.tot; // the selected buckets' keys (the next step's segment size)
            }
            plan_publish(o, st, pa.nsel, pa.status, pa.host_status);
        }
        if (o.status != 0) return;
        nsel = pa.nsel;
        b0 = o.b0;
        b1 = nsel > 1 ? o.b1 : -1;
    } else {
        if (status && *status != 0) return; // the device plan found no bucket path
        nsel = st->nsel;
        b0 = st->bsel[0];
        b1 = nsel > 1 ? st->bsel[1] : -1;
    }
    // one region per wave at a time (a region holds tens to hundreds of band
    // keys: the loads of 4 regions are in flight per block instead of one
    // region after another); matches gather in LDS, one global reservation
    // per block at the end (a wave writes straight to the segment if the LDS
    // buffer is full)
    __shared__ uint64_t sK[CB_LDS];
    __shared__ int sN, sValid; // reserved slots; the first slot a full buffer left unwritten
    __shared__ unsigned long long sBase;
    const uint64_t lo = st->lo_key;
    const double binv = st->binv;
    unsigned long long *ctr = reinterpret_cast<unsigned long long *>(seg);
    uint64_t *outk = seg + 1;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr int CU = 4; // loads in flight per lane
    if (threadIdx.x == 0) {
        sN = 0;
        sValid = CB_LDS;
    }
    __syncthreads();
    for (int64_t r = (int64_t)blockIdx.x * 4 + w; r < nreg; r += (int64_t)gridDim.x * 4) {
        int64_t cnt = counts ? (int64_t)counts[r] : cap;
        if (cnt > cap) cnt = cap;
        const uint64_t *kr = keys + r * cap;
        for (int64_t b = 0; b < cnt; b += 64 * CU) {
            uint64_t kk[CU];
#pragma unroll
            for (int u = 0; u < CU; ++u) {
                const int64_t e = b + u * 64 + lane;
                kk[u] = e < cnt ? kr[e] : 0;
            }
#pragma unroll
            for (int u = 0; u < CU; ++u) {
                const int64_t e = b + u * 64 + lane;
                const int kb = kbucket(kk[u], lo, binv);
                const bool m = e < cnt && (kb == b0 || kb == b1);
                const unsigned long long bal = __ballot(m);
                if (!bal) continue;
                const int c = __popcll(bal), off = __popcll(bal & ((1ull << lane) - 1ull));
                int base = 0;
                if (lane == 0) base = atomicAdd(&sN, c);
                base = __shfl(base, 0);
                if (base + c <= CB_LDS) {
                    if (m) sK[base + off] = kk[u];
                } else { // LDS buffer full: this wave reserves and writes directly
                    unsigned long long g = 0;
                    if (lane == 0) {
                        atomicMin(&sValid, base); // slots from base on stay unwritten
                        g = atomicAdd(ctr, (unsigned long long)c);
                    }
                    g = __shfl(g, 0);
                    if (m && g + off < (unsigned long long)seg_cap) outk[g + off] = kk[u];
                }
            }
        }
    }
    __syncthreads();
    const int m = min(sN, sValid);
    if (threadIdx.x == 0 && m) sBase = atomicAdd(ctr, (unsigned long long)m);
    __syncthreads();
    for (int e = threadIdx.x; e < m; e += 256) {
        const unsigned long long pos = sBase + e;
        if (pos < (unsigned long long)seg_cap) outk[pos] = sK[e];
    }
}

// Inclusive prefix sum of v over a 1024-thread block (wave shuffles + one
// LDS step over the 16 wave totals).  sW: 16 entries of scratch.
__device__ __forceinline__ unsigned long long block_scan_1024(unsigned long long v,
                                                              unsigned long long *sW)
{
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long t = __shfl_up(v, o);
        if (lane >= o) v += t;
    }
    if (lane == 63) sW[wv] = v;
    __syncthreads();
    if (wv == 0) {
        unsigned long long w = lane < 16 ? sW[lane] : 0ull;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            const unsigned long long t = __shfl_up(w, o);
            if (lane >= o) w += t;
        }
        if (lane < 16) sW[lane] = w;
    }
    __syncthreads();
    if (wv > 0) v += sW[wv - 1];
    __syncthreads(); // sW reusable
    return v;
}

// Exact selection over the gathered segments (one per rank): for each
// selection s, the rank[s]-th smallest key of bucket bsel[s].  Both
// selections advance together: radix passes (11-bit digits, LDS histograms,
// block scan) start below the common prefix of the selected buckets' keys
// (bits above it are equal for every key of a bucket), so a narrow bucket
// needs 2-3 passes.
// The last thread also maps the selected keys to the scale (k_finalize's
// arithmetic): scal = [a, med].
__device__ __forceinline__ void finalize_scale(const SelState *st, int navg, int src_lo, int src_hi,
                                               double logn, double *a_out, double *med_out);
__device__ __forceinline__ void select_small_body(SelState *st, const uint64_t *__restrict__ segs,
                                                  int nseg, int64_t seg_cap, int navg,
                                                  int src_lo, int src_hi, double logn,
                                                  double *__restrict__ scal,
                                                  const int *__restrict__ status,
                                                  uint64_t *__restrict__ trk)
{
    if (status && *status != 0) return; // the device plan found no bucket path
    __shared__ uint32_t sHist[2][RADIX];
    __shared__ unsigned long long sW[16];
    __shared__ unsigned long long sMn[2][16], sMx[2][16];
    __shared__ int sDigit[2];
    __shared__ unsigned long long sBelowD[2];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint64_t lo = st->lo_key;
    const double binv = st->binv;
    const int nsel = st->nsel;
    const int bs[2] = {st->bsel[0], nsel > 1 ? st->bsel[1] : st->bsel[0]};
    unsigned long long rank[2] = {st->rank[0], nsel > 1 ? st->rank[1] : st->rank[0]};
    {
        // Few keys (the usual case: a tracked or sampled bracket's bucket holds
        // tens to hundreds): gather each selected bucket's keys into LDS, sort
        // them (bitonic, padded to a power of two with ~0) and take the
        // rank-th -- exact, no radix passes.  Otherwise the radix path.
        // (Counting each key's rank over all others was O(n^2) on one CU:
        // 75 us at n = 1024.)
        constexpr int SEL_FAST = 1024;
        __shared__ uint64_t sKey[2][SEL_FAST];
        __shared__ int sN[2];
        if (tid < 2) sN[tid] = 0;
        __syncthreads();
        for (int g = 0; g < nseg; ++g) {
            const uint64_t *sg = segs + (int64_t)g * (seg_cap + 1);
            const int64_t cnt = min<int64_t>((int64_t)sg[0], seg_cap);
            for (int64_t e = tid; e < cnt; e += 1024) {
                const uint64_t key = sg[1 + e];
                const int kb = kbucket(key, lo, binv);
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    if (kb == bs[q]) {
                        const int pos = atomicAdd(&sN[q], 1);
                        if (pos < SEL_FAST) sKey[q][pos] = key;
                    }
            }
        }
        __syncthreads();
        const int n0 = sN[0], n1 = sN[1];
        if (n0 <= SEL_FAST && n1 <= SEL_FAST) {
            // register bitonic sort, one key per thread: partners within a
            // wave by shuffle (j < 64), across waves through LDS (j >= 64:
            // 10 of the 55 stages at 1024 keys, two barriers each)
            uint64_t sel[2];
            bool ok = true;
            const bool same = bs[1] == bs[0];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int nq = q ? n1 : n0;
                uint64_t *a = sKey[q];
                if (q == 1 && same) { // both order statistics in one bucket: sorted already
                    ok = ok && rank[1] < (unsigned long long)nq;
                    sel[1] = ok ? sKey[0][rank[1]] : 0ull;
                    break;
                }
                int p2 = 1;
                while (p2 < nq) p2 <<= 1;
                uint64_t x = tid < nq ? a[tid] : ~0ull; // padding sorts last
                for (int k = 2; k <= p2; k <<= 1)
                    for (int j = k >> 1; j > 0; j >>= 1) {
                        uint64_t y;
                        if (j >= 64) {
                            __syncthreads();
                            if (tid < p2) a[tid] = x;
                            __syncthreads();
                            y = tid < p2 ? a[tid ^ j] : x;
                        } else {
                            y = __shfl_xor(x, j);
                        }
                        const bool keep_min = ((tid & k) == 0) == ((tid & j) == 0);
                        x = keep_min ? (x < y ? x : y) : (x < y ? y : x);
                    }
                __syncthreads();
                if (tid < p2) a[tid] = x;
                __syncthreads();
                ok = ok && rank[q] < (unsigned long long)nq;
                sel[q] = ok ? a[rank[q]] : 0ull;
            }
            if (tid == 0) {
                if (!ok) st->error = 1; // rank outside the bucket (should not happen)
                st->prefix[0] = sel[0];
                if (nsel > 1) st->prefix[1] = sel[1];
                finalize_scale(st, navg, src_lo, src_hi, logn, scal, scal + 1);
                if (trk) {
                    trk[4] = sel[0];
                    trk[5] = nsel > 1 ? sel[1] : sel[0];
                    trk[6] = ok ? 0 : 1;
                }
            }
            return;
        }
    }
    // min / max key of each selected bucket
    uint64_t mn[2] = {~0ull, ~0ull}, mx[2] = {0, 0};
    for (int g = 0; g < nseg; ++g) {
        const uint64_t *sg = segs + (int64_t)g * (seg_cap + 1);
        const int64_t cnt = min<int64_t>((int64_t)sg[0], seg_cap);
        for (int64_t e = tid; e < cnt; e += 1024) {
            const uint64_t key = sg[1 + e];
            const int kb = kbucket(key, lo, binv);
#pragma unroll
            for (int q = 0; q < 2; ++q)
                if (kb == bs[q]) {
                    mn[q] = key < mn[q] ? key : mn[q];
                    mx[q] = key > mx[q] ? key : mx[q];
                }
        }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t a = __shfl_xor(mn[q], o), c = __shfl_xor(mx[q], o);
            mn[q] = a < mn[q] ? a : mn[q];
            mx[q] = c > mx[q] ? c : mx[q];
        }
        if (lane == 0) {
            sMn[q][wv] = mn[q];
            sMx[q][wv] = mx[q];
        }
    }
    __syncthreads();
    if (tid < 2) {
        uint64_t a = sMn[tid][0], c = sMx[tid][0];
        for (int w = 1; w < 16; ++w) {
            a = sMn[tid][w] < a ? sMn[tid][w] : a;
            c = sMx[tid][w] > c ? sMx[tid][w] : c;
        }
        sMn[tid][0] = a;
        sMx[tid][0] = c;
    }
    __syncthreads();
    int known = 0;
    uint64_t prefix[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const uint64_t diff = sMn[q][0] ^ sMx[q][0];
        const int kq = diff ? 64 - __clzll((long long)diff) : 0;
        known = kq > known ? kq : known;
    }
#pragma unroll
    for (int q = 0; q < 2; ++q)
        prefix[q] = known >= 64 ? 0ull : (sMn[q][0] & ~((1ull << known) - 1ull));
    bool err = false;
    while (known > 0) {
        const int width = known >= RADIX_BITS ? RADIX_BITS : known;
        const int shift = known - width;
        for (int e = tid; e < 2 * RADIX; e += 1024) (&sHist[0][0])[e] = 0;
        __syncthreads();
        for (int g = 0; g < nseg; ++g) {
            const uint64_t *sg = segs + (int64_t)g * (seg_cap + 1);
            const int64_t cnt = min<int64_t>((int64_t)sg[0], seg_cap);
            for (int64_t e = tid; e < cnt; e += 1024) {
                const uint64_t key = sg[1 + e];
                const int kb = kbucket(key, lo, binv);
                const uint32_t dg = (uint32_t)((key >> shift) & ((1u << width) - 1u));
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    if (kb == bs[q] && (known >= 64 || (key >> known) == (prefix[q] >> known)))
                        atomicAdd(&sHist[q][dg], 1u);
            }
        }
        __syncthreads();
        constexpr int PER = RADIX / 1024;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            unsigned long long loc = 0;
            for (int u = 0; u < PER; ++u) loc += sHist[q][tid * PER + u];
            const unsigned long long incl = block_scan_1024(loc, sW);
            const unsigned long long excl = incl - loc;
            if (tid == 0) sDigit[q] = -1;
            __syncthreads();
            if (rank[q] >= excl && rank[q] < incl) {
                unsigned long long c = excl;
                for (int u = 0; u < PER; ++u) {
                    const unsigned long long hv = sHist[q][tid * PER + u];
                    if (rank[q] < c + hv) {
                        sDigit[q] = tid * PER + u;
                        sBelowD[q] = c;
                        break;
                    }
                    c += hv;
                }
            }
            __syncthreads();
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            if (sDigit[q] < 0) {
                err = true;
            } else {
                prefix[q] |= (uint64_t)sDigit[q] << shift;
                rank[q] -= sBelowD[q];
            }
        }
        __syncthreads();
        if (err) break; // uniform: rank outside the bucket (the host checked; should not happen)
        known = shift;
    }
    if (tid == 0) {
        if (err) st->error = 1;
        st->prefix[0] = prefix[0];
        if (nsel > 1) st->prefix[1] = prefix[1];
        finalize_scale(st, navg, src_lo, src_hi, logn, scal, scal + 1);
        if (trk) { // the selected keys for the host's bracket tracking
            trk[4] = prefix[0];
            trk[5] = nsel > 1 ? prefix[1] : prefix[0];
            trk[6] = err ? 1 : 0;
        }
    }
}
// seq (speculative steps at timing level 0): after the selection, thread 0
// -- the one that wrote trk -- stores seq into trk[8], system-scope after its
// other stores; the host polls it instead of an event between this kernel
// and the next (an event record there cost a ~6 us dispatch gap per step).
// The plan's status in pinned memory was stored by an earlier kernel.
__global__ __launch_bounds__(1024) void k_select_small(SelState *st, const uint64_t *__restrict__ segs,
                                                      int nseg, int64_t seg_cap, int navg,
                                                      int src_lo, int src_hi, double logn,
                                                      double *__restrict__ scal,
                                                      const int *__restrict__ status,
                                                      uint64_t *__restrict__ trk, uint64_t seq)
{
    select_small_body(st, segs, nseg, seg_cap, navg, src_lo, src_hi, logn, scal, status, trk);
    if (seq && trk && threadIdx.x == 0) {
        __threadfence_system();
        *reinterpret_cast<volatile uint64_t *>(trk + 8) = seq;
    }
}

// One radix-select step: for each active selection find the digit holding
// its remaining rank, append it to the prefix, subtract the count below,
// zero the histogram and advance to the next digit.
// make_bracket (the sample's last pass): also the candidate bracket [lo_key,
// hi_key) from the buckets of selection 0 (lower edge) and 1 (upper edge).
__global__ __launch_bounds__(256) void k_select_scan(SelState *st, unsigned long long *ghist,
                                                    int make_bracket, unsigned long long *bzero)
{
    if (make_bracket && bzero) // the coming collect pass's bucket counts
        for (int e = threadIdx.x; e < NBK; e += 256) bzero[e] = 0;
    __shared__ unsigned long long sPart[256];
    __shared__ int sDigit;
    __shared__ unsigned long long sBelowD;
    const int tid = threadIdx.x;
    const int nsel = st->nsel, shift = st->shift, width = st->width;
    constexpr int PER = RADIX / 256;
    for (int s = 0; s < nsel; ++s) {
        const unsigned long long *h = ghist + s * RADIX;
        unsigned long long loc = 0;
        for (int q = 0; q < PER; ++q) loc += h[tid * PER + q];
        sPart[tid] = loc;
        if (tid == 0) sDigit = -1;
        __syncthreads();
        // inclusive scan over 256 partials (Hillis-Steele)
        for (int o = 1; o < 256; o <<= 1) {
            unsigned long long v = tid >= o ? sPart[tid - o] : 0ull;
            __syncthreads();
            sPart[tid] += v;
            __syncthreads();
        }
        const unsigned long long rank = st->rank[s];
        const unsigned long long excl = tid ? sPart[tid - 1] : 0ull;
        if (rank >= excl && rank < sPart[tid]) {
            unsigned long long c = excl;
            for (int q = 0; q < PER; ++q) {
                const unsigned long long hv = h[tid * PER + q];
                if (rank < c + hv) {
                    sDigit = tid * PER + q;
                    sBelowD = c;
                    break;
                }
                c += hv;
            }
        }
        __syncthreads();
        if (tid == 0) {
            if (sDigit < 0) {
                st->error = 1;
            } else {
                st->prefix[s] |= (uint64_t)sDigit << shift;
                st->rank[s] = rank - sBelowD;
            }
        }
        __syncthreads();
    }
    for (int e = tid; e < 2 * RADIX; e += 256) ghist[e] = 0;
    if (tid == 0) {
        st->pass += 1;
        const int nshift = shift - RADIX_BITS;
        st->shift = nshift >= 0 ? nshift : 0;
        st->width = nshift >= 0 ? RADIX_BITS : shift;
        (void)width;
        if (make_bracket) {
            const int sh = st->shift + st->width; // bits below the resolved digits
            st->lo_key = st->prefix[0];
            const uint64_t top = st->prefix[1] + (sh >= 64 ? 0ull : (1ull << sh));
            st->hi_key = (top < st->prefix[1]) ? ~0ull : top;
            st->binv = (double)NBK / (double)(st->hi_key - st->lo_key);
        }
    }
}

// Collect outputs -> cnt, in one launch.  Blocks 0 .. NBK/64-1: the
// key-range bucket counts cnt[3 + e] = sum_b bpart[b][e] (zero without
// bpart; integer sums in fixed order).  The last block: cnt[0] = below,
// cnt[1] = candidates (true count), cnt[2] = overflowed regions (all sums, so
// one all-reduce serves every rank), cnt[CNT_LO..CNT_HI] = the bracket for
// the host.
constexpr int BSUM_SLICES = 16; // partial slices per 64-bucket group (k_counts_reduce)
__global__ __launch_bounds__(256) void k_counts_reduce(const unsigned long long *__restrict__ below,
                                                      const uint32_t *__restrict__ counts,
                                                      int64_t nblk, int64_t cap,
                                                      const SelState *__restrict__ st,
                                                      const uint32_t *__restrict__ bpart,
                                                      int64_t nbpart,
                                                      unsigned long long *__restrict__ cnt,
                                                      uint64_t *__restrict__ seg_zero)
{
    __shared__ unsigned long long s0[256], s1[256], s2[256];
    if ((int)blockIdx.x < NBK / 64 * BSUM_SLICES) {
        // bucket group blockIdx % (NBK/64), partial slice blockIdx / (NBK/64);
        // cnt[3 .. 3 + NBK) was zeroed this step (k_center / the bracket scan)
        if (!bpart) return;
        const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
        const int grp = blockIdx.x % (NBK / 64), sl = blockIdx.x / (NBK / 64);
        const int e = grp * 64 + lane;
        const int64_t per = (nbpart + BSUM_SLICES - 1) / BSUM_SLICES;
        const int64_t p0 = sl * per, p1 = min(nbpart, p0 + per);
        unsigned long long acc = 0;
        for (int64_t b0 = p0 + g; b0 < p1; b0 += 32) {
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t b = b0 + 4 * u;
                v[u] = b < p1 ? bpart[b * NBK + e] : 0u;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += v[u];
        }
        s0[threadIdx.x] = acc;
        __syncthreads();
        if (g == 0) {
            const unsigned long long t = s0[lane] + s0[64 + lane] + s0[128 + lane] + s0[192 + lane];
            if (t) atomicAdd(&cnt[3 + e], t);
        }
        return;
    }
    unsigned long long b = 0, c = 0, o = 0;
    for (int64_t e = threadIdx.x; e < nblk; e += 256) {
        b += below[e];
        c += counts[e];
        o += (counts[e] > cap) ? 1ull : 0ull;
    }
    s0[threadIdx.x] = b;
    s1[threadIdx.x] = c;
    s2[threadIdx.x] = o;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k) {
            s0[threadIdx.x] += s0[threadIdx.x + k];
            s1[threadIdx.x] += s1[threadIdx.x + k];
            s2[threadIdx.x] += s2[threadIdx.x + k];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        cnt[0] = s0[0];
        cnt[1] = s1[0];
        cnt[2] = s2[0];
        cnt[CNT_LO] = st->lo_key;
        cnt[CNT_HI] = st->hi_key;
        if (seg_zero) seg_zero[0] = 0; // the speculative compaction's counter
    }
}

// med = (sqrt(u_lo) + sqrt(u_hi)) / 2 (or the single middle value);
// a = ln(n) / med^2  (GaussianRBFKernel.hpp:187, ComputeMedian :222-254).
// src_lo / src_hi: selection slot holding each order statistic, -1 for a
// diagonal zero of the full n^2 list.
__device__ __forceinline__ void finalize_scale(const SelState *st, int navg, int src_lo, int src_hi,
                                               double logn, double *a_out, double *med_out)
{
    const double u0 =
        src_lo < 0 ? 0.0 : sqrt(__longlong_as_double((long long)st->prefix[src_lo]));
    double med;
    if (navg == 2) {
        const double u1 =
            src_hi < 0 ? 0.0 : sqrt(__longlong_as_double((long long)st->prefix[src_hi]));
        med = (u0 + u1) / 2.0;
    } else {
        med = u0;
    }
    *med_out = med;
    *a_out = logn / (med * med);
}
__global__ void k_finalize(const SelState *st, int navg, int src_lo, int src_hi, double logn,
                           double *a_out, double *med_out)
{
    finalize_scale(st, navg, src_lo, src_hi, logn, a_out, med_out);
}

// ===================================================== row-stream kernels ==
//
// gfx950 runs f64 MFMA and f64 VALU on one shared pipeline (tools/ubench_f64:
// ~64 TF MFMA alone, ~68 TF VALU alone, ~70 TF mixed), and these loops are
// instruction-issue bound (rocprof: one instruction per SIMD per 4 cycles,
// whatever its type), so for small d the phi pass minimises instructions
// per pair instead of using MFMA:
//
//   lane = R particle rows i (pre-scaled by 8192 a log2e), column particle j
//   wave-uniform: its record arrives in LDS by DMA (per-wave double-buffered
//   chunks) and is read with broadcast ds_read_b128.
//   per (i, j):  u    add + d FMA    (u = 4096 log2 K_ij, Gram form on centred x)
//                2^(u/4096)          4096-entry LDS table x degree-2 form, ldexp
//                acc  d FMA + 1      (sum_j K_ij V_j, sum_j K_ij)
//   3d + 9 f64 ops per ordered pair (d = 8: 33 incl. the integer ops).
// Columns are split over S workgroups (partials reduced by k_phi_reduce in a
// fixed order, so results are deterministic).

// 2^(i/256), i = 0..255, correctly rounded (tools/make_exp_table.py)
__constant__ double EXP2_TAB256[256] = {
    0x1.0000000000000p+0, 0x1.00b1afa5abcbfp+0, 0x1.0163da9fb3335p+0, 0x1.02168143b0281p+0,
    0x1.02c9a3e778061p+0, 0x1.037d42e11bbccp+0, 0x1.04315e86e7f85p+0, 0x1.04e5f72f654b1p+0,
    0x1.059b0d3158574p+0, 0x1.0650a0e3c1f89p+0, 0x1.0706b29ddf6dep+0, 0x1.07bd42b72a836p+0,
    0x1.0874518759bc8p+0, 0x1.092bdf66607e0p+0, 0x1.09e3ecac6f383p+0, 0x1.0a9c79b1f3919p+0,
    0x1.0b5586cf9890fp+0, 0x1.0c0f145e46c85p+0, 0x1.0cc922b7247f7p+0, 0x1.0d83b23395decp+0,
    0x1.0e3ec32d3d1a2p+0, 0x1.0efa55fdfa9c5p+0, 0x1.0fb66affed31bp+0, 0x1.1073028d7233ep+0,
    0x1.11301d0125b51p+0, 0x1.11edbab5e2ab6p+0, 0x1.12abdc06c31ccp+0, 0x1.136a814f204abp+0,
    0x1.1429aaea92de0p+0, 0x1.14e95934f312ep+0, 0x1.15a98c8a58e51p+0, 0x1.166a45471c3c2p+0,
    0x1.172b83c7d517bp+0, 0x1.17ed48695bbc0p+0, 0x1.18af9388c8deap+0, 0x1.1972658375d2fp+0,
    0x1.1a35beb6fcb75p+0, 0x1.1af99f8138a1cp+0, 0x1.1bbe084045cd4p+0, 0x1.1c82f95281c6bp+0,
    0x1.1d4873168b9aap+0, 0x1.1e0e75eb44027p+0, 0x1.1ed5022fcd91dp+0, 0x1.1f9c18438ce4dp+0,
    0x1.2063b88628cd6p+0, 0x1.212be3578a819p+0, 0x1.21f49917ddc96p+0, 0x1.22bdda27912d1p+0,
    0x1.2387a6e756238p+0, 0x1.2451ffb82140ap+0, 0x1.251ce4fb2a63fp+0, 0x1.25e85711ece75p+0,
    0x1.26b4565e27cddp+0, 0x1.2780e341ddf29p+0, 0x1.284dfe1f56381p+0, 0x1.291ba7591bb70p+0,
    0x1.29e9df51fdee1p+0, 0x1.2ab8a66d10f13p+0, 0x1.2b87fd0dad990p+0, 0x1.2c57e39771b2fp+0,
    0x1.2d285a6e4030bp+0, 0x1.2df961f641589p+0, 0x1.2ecafa93e2f56p+0, 0x1.2f9d24abd886bp+0,
    0x1.306fe0a31b715p+0, 0x1.31432edeeb2fdp+0, 0x1.32170fc4cd831p+0, 0x1.32eb83ba8ea32p+0,
    0x1.33c08b26416ffp+0, 0x1.3496266e3fa2dp+0, 0x1.356c55f929ff1p+0, 0x1.36431a2de883bp+0,
    0x1.371a7373aa9cbp+0, 0x1.37f26231e754ap+0, 0x1.38cae6d05d866p+0, 0x1.39a401b7140efp+0,
    0x1.3a7db34e59ff7p+0, 0x1.3b57fbfec6cf4p+0, 0x1.3c32dc313a8e5p+0, 0x1.3d0e544ede173p+0,
    0x1.3dea64c123422p+0, 0x1.3ec70df1c5175p+0, 0x1.3fa4504ac801cp+0, 0x1.40822c367a024p+0,
    0x1.4160a21f72e2ap+0, 0x1.423fb2709468ap+0, 0x1.431f5d950a897p+0, 0x1.43ffa3f84b9d4p+0,
    0x1.44e086061892dp+0, 0x1.45c2042a7d232p+0, 0x1.46a41ed1d0057p+0, 0x1.4786d668b3237p+0,
    0x1.486a2b5c13cd0p+0, 0x1.494e1e192aed2p+0, 0x1.4a32af0d7d3dep+0, 0x1.4b17dea6db7d7p+0,
    0x1.4bfdad5362a27p+0, 0x1.4ce41b817c114p+0, 0x1.4dcb299fddd0dp+0, 0x1.4eb2d81d8abffp+0,
    0x1.4f9b2769d2ca7p+0, 0x1.508417f4531eep+0, 0x1.516daa2cf6642p+0, 0x1.5257de83f4eefp+0,
    0x1.5342b569d4f82p+0, 0x1.542e2f4f6ad27p+0, 0x1.551a4ca5d920fp+0, 0x1.56070dde910d2p+0,
    0x1.56f4736b527dap+0, 0x1.57e27dbe2c4cfp+0, 0x1.58d12d497c7fdp+0, 0x1.59c0827ff07ccp+0,
    0x1.5ab07dd485429p+0, 0x1.5ba11fba87a03p+0, 0x1.5c9268a5946b7p+0, 0x1.5d84590998b93p+0,
    0x1.5e76f15ad2148p+0, 0x1.5f6a320dceb71p+0, 0x1.605e1b976dc09p+0, 0x1.6152ae6cdf6f4p+0,
    0x1.6247eb03a5585p+0, 0x1.633dd1d1929fdp+0, 0x1.6434634ccc320p+0, 0x1.652b9febc8fb7p+0,
    0x1.6623882552225p+0, 0x1.671c1c70833f6p+0, 0x1.68155d44ca973p+0, 0x1.690f4b19e9538p+0,
    0x1.6a09e667f3bcdp+0, 0x1.6b052fa75173ep+0, 0x1.6c012750bdabfp+0, 0x1.6cfdcddd47645p+0,
    0x1.6dfb23c651a2fp+0, 0x1.6ef9298593ae5p+0, 0x1.6ff7df9519484p+0, 0x1.70f7466f42e87p+0,
    0x1.71f75e8ec5f74p+0, 0x1.72f8286ead08ap+0, 0x1.73f9a48a58174p+0, 0x1.74fbd35d7cbfdp+0,
    0x1.75feb564267c9p+0, 0x1.77024b1ab6e09p+0, 0x1.780694fde5d3fp+0, 0x1.790b938ac1cf6p+0,
    0x1.7a11473eb0187p+0, 0x1.7b17b0976cfdbp+0, 0x1.7c1ed0130c132p+0, 0x1.7d26a62ff86f0p+0,
    0x1.7e2f336cf4e62p+0, 0x1.7f3878491c491p+0, 0x1.80427543e1a12p+0, 0x1.814d2add106d9p+0,
    0x1.82589994cce13p+0, 0x1.8364c1eb941f7p+0, 0x1.8471a4623c7adp+0, 0x1.857f4179f5b21p+0,
    0x1.868d99b4492edp+0, 0x1.879cad931a436p+0, 0x1.88ac7d98a6699p+0, 0x1.89bd0a478580fp+0,
    0x1.8ace5422aa0dbp+0, 0x1.8be05bad61778p+0, 0x1.8cf3216b5448cp+0, 0x1.8e06a5e0866d9p+0,
    0x1.8f1ae99157736p+0, 0x1.902fed0282c8ap+0, 0x1.9145b0b91ffc6p+0, 0x1.925c353aa2fe2p+0,
    0x1.93737b0cdc5e5p+0, 0x1.948b82b5f98e5p+0, 0x1.95a44cbc8520fp+0, 0x1.96bdd9a7670b3p+0,
    0x1.97d829fde4e50p+0, 0x1.98f33e47a22a2p+0, 0x1.9a0f170ca07bap+0, 0x1.9b2bb4d53fe0dp+0,
    0x1.9c49182a3f090p+0, 0x1.9d674194bb8d5p+0, 0x1.9e86319e32323p+0, 0x1.9fa5e8d07f29ep+0,
    0x1.a0c667b5de565p+0, 0x1.a1e7aed8eb8bbp+0, 0x1.a309bec4a2d33p+0, 0x1.a42c980460ad8p+0,
    0x1.a5503b23e255dp+0, 0x1.a674a8af46052p+0, 0x1.a799e1330b358p+0, 0x1.a8bfe53c12e59p+0,
    0x1.a9e6b5579fdbfp+0, 0x1.ab0e521356ebap+0, 0x1.ac36bbfd3f37ap+0, 0x1.ad5ff3a3c2774p+0,
    0x1.ae89f995ad3adp+0, 0x1.afb4ce622f2ffp+0, 0x1.b0e07298db666p+0, 0x1.b20ce6c9a8952p+0,
    0x1.b33a2b84f15fbp+0, 0x1.b468415b749b1p+0, 0x1.b59728de5593ap+0, 0x1.b6c6e29f1c52ap+0,
    0x1.b7f76f2fb5e47p+0, 0x1.b928cf22749e4p+0, 0x1.ba5b030a1064ap+0, 0x1.bb8e0b79a6f1fp+0,
    0x1.bcc1e904bc1d2p+0, 0x1.bdf69c3f3a207p+0, 0x1.bf2c25bd71e09p+0, 0x1.c06286141b33dp+0,
    0x1.c199bdd85529cp+0, 0x1.c2d1cd9fa652cp+0, 0x1.c40ab5fffd07ap+0, 0x1.c544778fafb22p+0,
    0x1.c67f12e57d14bp+0, 0x1.c7ba88988c933p+0, 0x1.c8f6d9406e7b5p+0, 0x1.ca3405751c4dbp+0,
    0x1.cb720dcef9069p+0, 0x1.ccb0f2e6d1675p+0, 0x1.cdf0b555dc3fap+0, 0x1.cf3155b5bab74p+0,
    0x1.d072d4a07897cp+0, 0x1.d1b532b08c968p+0, 0x1.d2f87080d89f2p+0, 0x1.d43c8eacaa1d6p+0,
    0x1.d5818dcfba487p+0, 0x1.d6c76e862e6d3p+0, 0x1.d80e316c98398p+0, 0x1.d955d71ff6075p+0,
    0x1.da9e603db3285p+0, 0x1.dbe7cd63a8315p+0, 0x1.dd321f301b460p+0, 0x1.de7d5641c0658p+0,
    0x1.dfc97337b9b5fp+0, 0x1.e11676b197d17p+0, 0x1.e264614f5a129p+0, 0x1.e3b333b16ee12p+0,
    0x1.e502ee78b3ff6p+0, 0x1.e653924676d76p+0, 0x1.e7a51fbc74c83p+0, 0x1.e8f7977cdb740p+0,
    0x1.ea4afa2a490dap+0, 0x1.eb9f4867cca6ep+0, 0x1.ecf482d8e67f1p+0, 0x1.ee4aaa2188510p+0,
    0x1.efa1bee615a27p+0, 0x1.f0f9c1cb6412ap+0, 0x1.f252b376bba97p+0, 0x1.f3ac948dd7274p+0,
    0x1.f50765b6e4540p+0, 0x1.f6632798844f8p+0, 0x1.f7bfdad9cbe14p+0, 0x1.f91d802243c89p+0,
    0x1.fa7c1819e90d8p+0, 0x1.fbdba3692d514p+0, 0x1.fd3c22b8f71f1p+0, 0x1.fe9d96b2a23d9p+0};

// 2^(u/256) for u <= ~0: u = k + f, |f| <= 1/2, 2^(u/256) = 2^(k>>8) 2^((k&255)/256) 2^(f/256);
// 2^(f/256) = e^r, r = f ln2/256, |r| <= 1.36e-3, by its degree-4 Taylor
// polynomial (remainder r^5/5! < 0.35 ulp; <= ~2 ulp overall).  9 fp64 ops.
__device__ __forceinline__ double exp2_256_poly(double f)
{
    double p = 0x1.3b2ab6fba4e77p-39;
    p = fma(p, f, 0x1.c6b08d704a0c0p-29);
    p = fma(p, f, 0x1.ebfbdff82c58fp-19);
    p = fma(p, f, 0x1.62e42fefa39efp-9);
    return fma(p, f, 1.0);
}
__device__ __forceinline__ double exp2_256(double u, const double *tab)
{
    const double k = __builtin_rint(u);
    const double f = u - k;
    const int ki = (int)k;
    return __builtin_ldexp(exp2_256_poly(f) * tab[ki & 255], ki >> 8);
}

// Row-stream form: 2^(u/4096) for u <= ~0, u = k + f, |f| <= 1/2:
// 2^(k>>12) 2^((k&4095)/4096) 2^(f/4096), the last by the levelled degree-2
// form 1 + c1 f + c2 f^2 (tools/make_exp_table.py coeffs4096: relative error
// <= 2.6e-14, i.e. phi_hat within 2.6e-14 max|V| of the exact-exp sum, far
// inside the 1e-10 bound).  Two FMA fewer per pair than exp2_256 (32 KiB table).
__device__ __forceinline__ double exp2_4096_poly(double f)
{
    return fma(fma(0x1.ebfbdff82c58fp-27, f, 0x1.62e42ff4f7b0ap-13), f, 1.0);
}

constexpr int CH_PHI = 16; // columns per LDS chunk of the phi row stream
// the 8-wave row stream (kind 2): 8 waves, columns split over the 8 waves
constexpr int T8K_NW = 8, T8K_WC = 8;
constexpr int EXP_TB = 4096; // row-stream exp table entries
// Biased exponent (the 8-wave kernel, TABN = 8192): u' = u + EXP_UB >= 0 on
// both forms (folded u >= -1001 x 4096, plain |u| <= 1000 x 4096), so
// floor(u') = the truncating conversion and u' - floor(u') = v_fract_f64:
// the range reduction takes 2 VALU instead of 3 (rint, sub, cvt).  The table
// entries carry -(EXP_QB << 20) in their high word to undo the 2^EXP_QB.
// c_j + EXP_UB is stored in the record's slot 2d + 1 (k_prep_rec).
constexpr int EXP_QB = 1002;
constexpr double EXP_UB = (double)EXP_QB * EXP_TB;

// rec_j = [xc_j (D) | V_j = G_j - 2a xc_j (D) | c_j = -4096 a log2e |xc_j|^2 | 0 ...],
// stride phi_rec_stride(D) = roundup(2D+1, 8) doubles, so CH_PHI records are
// a whole number of 1 KiB LDS-DMA pieces.
template <int D> struct RecLayout {
    static constexpr int RS = phi_rec_stride(D);
};

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_void;

// Copy BYTES (multiple of 1 KiB) from global to this wave's LDS buffer with
// global_load_lds_dwordx4 (one 1 KiB piece per wave instruction; counted by
// vmcnt, no VGPR destination).
template <int BYTES>
__device__ __forceinline__ void dma_to_lds(const char *gsrc, char *ldst, int lane)
{
#pragma unroll
    for (int p = 0; p < BYTES / 1024; ++p)
        __builtin_amdgcn_global_load_lds((gbl_void *)(gsrc + p * 1024 + lane * 16),
                                         (lds_void *)(ldst + p * 1024), 16, 0, 0);
}

// s_waitcnt vmcnt(N) through the intrinsic (gfx9 encoding: vmcnt[3:0] in bits
// 3:0, vmcnt[5:4] in 15:14, expcnt/lgkmcnt left at their maxima), so the
// compiler's own wait insertion sees it and does not add a vmcnt(0) of its own
// at the first use of registers loaded before the wait.
template <int N> __device__ __forceinline__ void wait_vmcnt()
{
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}

// LDS accesses the compiler does not see: used for the collect pass's key
// staging area, which no LDS DMA ever targets.  A compiler-visible LDS store
// there would make it drain every in-flight column DMA first (it cannot prove
// the two do not alias).  The caller waits (lgkm_wait) before reading back.
__device__ __forceinline__ void lds_store_u64(const uint64_t *p, uint64_t v)
{
    const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const uint64_t *)p;
    asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_add_u32(const uint32_t *p, uint32_t v)
{
    const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const uint32_t *)p;
    asm volatile("ds_add_u32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
// Loads: the destination registers are only valid after lgkmcnt drains and the
// compiler does not know that, so every load helper waits inside the same asm
// statement (early-clobber outputs keep the address registers intact).
__device__ __forceinline__ uint32_t lds_addr(const void *p)
{
    return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char *)p;
}
// v[t] = p[t * 64] for t < 8 (one wave's 512-key staging row)
__device__ __forceinline__ void lds_load8_u64_sync(const uint64_t *p, uint64_t (&v)[8])
{
    asm volatile("ds_read_b64 %0, %8\n\t"
                 "ds_read_b64 %1, %8 offset:512\n\t"
                 "ds_read_b64 %2, %8 offset:1024\n\t"
                 "ds_read_b64 %3, %8 offset:1536\n\t"
                 "ds_read_b64 %4, %8 offset:2048\n\t"
                 "ds_read_b64 %5, %8 offset:2560\n\t"
                 "ds_read_b64 %6, %8 offset:3072\n\t"
                 "ds_read_b64 %7, %8 offset:3584\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]),
                   "=&v"(v[6]), "=&v"(v[7])
                 : "v"(lds_addr(p))
                 : "memory");
}
__device__ __forceinline__ void lgkm_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ uint64_t lds_load_u64_sync(const uint64_t *p)
{
    uint64_t v;
    asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(v) : "v"(lds_addr(p)) : "memory");
    return v;
}

// rec_j = [xc_j | G_j - 2a xc_j | -4096 a log2e |xc_j|^2 | 0..], one thread per
// element (coalesced stores of the np x RS array).
__global__ void k_prep_rec(const double *__restrict__ xc, const double *__restrict__ G,
                           const double *__restrict__ nrm, const double *__restrict__ a_ptr,
                           int64_t n, int64_t np, int d, int KP, int RS, double *__restrict__ rec)
{
    const double a = *a_ptr;
    const int64_t tot = np * RS;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = e / RS;
        const int k = (int)(e - j * RS);
        double v = 0.0;
        if (j < n) {
            if (k < d)
                v = xc[j * KP + k];
            else if (k < 2 * d)
                v = G[j * d + (k - d)] - 2.0 * a * xc[j * KP + (k - d)];
            else if (k == 2 * d)
                v = -4096.0 * a * LOG2E * nrm[j];
            else if (k == 2 * d + 1)
                v = -4096.0 * a * LOG2E * nrm[j] + EXP_UB;
        }
        rec[e] = v;
    }
}

// The row stream's LDS table holds T[m] = 2^(m/4096) with its high word
// biased by -(m << 8) (integer arithmetic mod 2^32).  For u = 4096 q + m
// (m = u & 4095) the high word plus (u << 8) is T[m]'s high word plus
// (q << 20): 2^q T[m] with ONE v_lshl_add_u32 -- in place of the shift and
// v_ldexp_f64 -- valid while 1023 + q stays inside the exponent field
// (callers keep q in [-1001, 1000]).
__device__ __forceinline__ double tab_biased(double t, int m)
{
    return __hiloint2double(__double2hiint(t) - (m << 8), __double2loint(t));
}
__device__ __forceinline__ double tab_scale(double tb, int ki)
{
    return __hiloint2double(__double2hiint(tb) + (ki << 8), __double2loint(tb));
}
constexpr double EXP_U_CLAMP = 1000.0 * EXP_TB; // |u| bound of the clamped (plain) form
// 2^(f/4096) on f in [0, 1) (minimax, relative error 2.54e-14; tools/exp_poly_fit.py)
__device__ __forceinline__ double exp2_4096_poly01(double f)
{
    return fma(fma(0x1.ec0687f62a7d5p-27, f, 0x1.62e42fdfa8275p-13), f, 0x1.0000000000071p+0);
}

// One column record of the phi row stream, held in registers.
// CS: the slot of c_j (2D: c_j; 2D + 1: c_j + EXP_UB, the biased-exponent
// kernels' folded form)
template <int D> struct ColRec {
    double x[D], v[D], c;
    template <int CS = 2 * D> __device__ __forceinline__ void load(const double *rj)
    {
#pragma unroll
        for (int k = 0; k < D; ++k) {
            x[k] = rj[k];
            v[k] = rj[D + k];
        }
        c = rj[CS];
    }
};

// acc_i += K_ij [V_j, 1] for the lane's R rows against one column j.
// FOLD: the row term c_i is left out of u (one add fewer per pair) and the
// row's sums are scaled by 2^(c_i/4096) once at the end (k_phi_rows); the
// kernel takes it only where u provably stays inside [-1001, 400] x 4096, so
// no clamp either.  Plain form: u clamped to +-EXP_U_CLAMP (K within
// [2^-1000, 2^1000] instead of [0, inf]: below any fp64 sum that holds the
// diagonal K_ii = 1).
// Byte offset of table entry (ki mod 8192) in ONE instruction: the 16-bit
// shift zeroes the destination's high half on gfx9 (tools/check_b16.hip
// checks it on the device), so (ki << 3) & 0xffff needs no separate mask.
__device__ __forceinline__ uint32_t tab8k_offset(int ki)
{
    uint32_t a;
    asm("v_lshlrev_b16 %0, 3, %1" : "=v"(a) : "v"(ki));
    return a;
}

// TABN = 8192: the biased exponent (EXP_UB): q.c is c_j + EXP_UB (folded)
// and ci is c_i + EXP_UB (plain form), so u >= 0 here.
template <int D, int R, bool FOLD, int TABN = EXP_TB>
__device__ __forceinline__ void phi_rows_pair(const ColRec<D> &q, const double (&xs)[R][D],
                                              const double (&ci)[R], double (&acc)[R][D],
                                              double (&acc1)[R], const double *tab)
{
    constexpr bool BIAS = TABN == 8192;
    // the R rows' chains interleaved (independent FMAs back to back)
    double u[R], K[R];
#pragma unroll
    for (int r = 0; r < R; ++r) u[r] = FOLD ? q.c : ci[r] + q.c;
#pragma unroll
    for (int k = 0; k < D; ++k)
#pragma unroll
        for (int r = 0; r < R; ++r) u[r] = fma(xs[r][k], q.x[k], u[r]);
    if constexpr (!FOLD) {
        constexpr double lo = BIAS ? EXP_UB - EXP_U_CLAMP : -EXP_U_CLAMP;
        constexpr double hi = BIAS ? EXP_UB + EXP_U_CLAMP : EXP_U_CLAMP;
#pragma unroll
        for (int r = 0; r < R; ++r) u[r] = fmin(fmax(u[r], lo), hi);
    }
    // exp2_256 in stages: the R table reads are issued together and their
    // LDS latency hides behind the R polynomials
    double f[R], T[R];
    int ki[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if constexpr (BIAS) {
            f[r] = __builtin_amdgcn_fract(u[r]); // u >= 0: u - floor(u)
            ki[r] = (int)u[r];                    // = floor(u)
            T[r] = *reinterpret_cast<const double *>(reinterpret_cast<const char *>(tab) + tab8k_offset(ki[r]));
        } else {
            const double k = __builtin_rint(u[r]);
            f[r] = u[r] - k;
            ki[r] = (int)k;
            T[r] = tab[ki[r] & (EXP_TB - 1)];
        }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < R; ++r) K[r] = BIAS ? exp2_4096_poly01(f[r]) : exp2_4096_poly(f[r]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < R; ++r) K[r] = K[r] * tab_scale(T[r], ki[r]);
#pragma unroll
    for (int k = 0; k < D; ++k)
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r][k] = fma(K[r], q.v[k], acc[r][k]);
#pragma unroll
    for (int r = 0; r < R; ++r) acc1[r] += K[r];
}

// sgn (matrix scale, M = L S L^T): the row coordinates are scaled by S so
// the pair term is z_i^T S z_j; nullptr = the isotropic scale (S = I).
// NW waves per work-group; TABN = 4096 (the 32 KiB table, 4 waves) or 8192
// (a 64 KiB table -- two octaves, T[m + 4096] = 2 T[m] exactly -- whose
// address needs no mask, tab8k_offset; 8 waves share it so the LDS still
// fits 8 waves per CU).
// WC: the waves of a work-group split its column range WC ways (NW / WC row
// groups of 64 R rows): their partial sums are added in LDS in wave order
// before one partial per work-group goes out -- WC times fewer partials (HBM
// writes here, reads in k_phi_reduce) for the same number of waves.
// LDS bytes of the row stream's work-group: per-wave double-buffered column
// chunks, then the 2^(i/4096) table
template <int D, int NW, int TABN> constexpr int phi_rows_lds()
{
    return NW * 2 * (CH_PHI * RecLayout<D>::RS * 8) + TABN * 8;
}

// The row stream's work-group `bid` of a grid of (row groups) x S blocks, on
// the caller's LDS (phi_rows_lds bytes): k_phi_rows, and k_phi_sym when the
// symmetric form does not apply (its hand-over, symok = 0).
template <int D, int R, int NW, int TABN, int WC>
__device__ __forceinline__ void phi_rows_body(char *smem, int64_t bid, const double *__restrict__ rec,
                                              const double *__restrict__ a_ptr, int64_t row0, int64_t nrows,
                                              int64_t n, int S, double *__restrict__ part, int64_t ldp,
                                              const double *__restrict__ sgn,
                                              const unsigned long long *__restrict__ nmax_bits)
{
    constexpr int RS = RecLayout<D>::RS;
    constexpr int CHB = CH_PHI * RS * 8; // bytes per column chunk (multiple of 1 KiB)
    // register double buffer of the column record only where it fits without
    // spilling (row state R(2D+2) + two records 2(2D+1) doubles)
    constexpr bool PIPE = (R * (2 * D + 2) + 2 * (2 * D + 1)) * 2 <= 232;
    double *tab = reinterpret_cast<double *>(smem + NW * 2 * CHB);
#pragma unroll
    for (int e = 0; e < TABN / (NW * 64); ++e) {
        const int m = e * NW * 64 + threadIdx.x;
        const double t = EXP2_TAB4096[m & (EXP_TB - 1)];
        const double tb = tab_biased(m >= EXP_TB ? 2.0 * t : t, m);
        // TABN = 8192: also -(EXP_QB << 20), undoing the exponent bias
        tab[m] = TABN == 8192 ? __hiloint2double(__double2hiint(tb) - (EXP_QB << 20), __double2loint(tb)) : tb;
    }
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    char *wbuf = smem + w * 2 * CHB;
    static_assert(NW % WC == 0, "WC must divide NW");
    constexpr int WR = NW / WC; // row groups per work-group
    const int wr = w % WR, wc = w / WR;
    const int64_t iblk = bid / S;
    const int s = (int)(bid - iblk * S);
    const int64_t rbase = iblk * (WR * 64 * R) + wr * (64 * R); // local row of this wave's lane 0
    // u_ij = c_i + c_j + 8192 a log2e xc_i.xc_j = -4096 a log2e |xc_i - xc_j|^2;
    // the row coordinates are pre-scaled by 8192 a log2e
    const double alpha = 8192.0 * LOG2E * (*a_ptr);

    double xs[R][D], ci[R], acc[R][D], acc1[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int64_t li = rbase + 64 * r + lane;
        if (li >= nrows) li = nrows - 1; // padding lanes recompute a valid row
        const double *ri = rec + (row0 + li) * RS;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            xs[r][k] = (sgn ? alpha * sgn[k] : alpha) * ri[k];
            acc[r][k] = 0.0;
        }
        ci[r] = ri[2 * D];
        acc1[r] = 0.0;
    }

    // Column records stream through two LDS chunk buffers: the DMA of chunk
    // c+1 is in flight (vmcnt) while chunk c is computed; every lane reads the
    // same record (LDS broadcast), one column ahead of its use so the LDS
    // latency overlaps the previous column's arithmetic.  rec has >= 64 padded
    // rows past n, so whole chunks may be copied; the look-ahead read past a
    // chunk stays inside smem and is discarded.
    // column split of this wave: s (the work-group's) refined WC ways
    const int64_t ST = (int64_t)S * WC, sw = (int64_t)s * WC + wc;
    const int64_t j0 = n * sw / ST, j1 = n * (sw + 1) / ST;
    const int64_t nch = (j1 - j0 + CH_PHI - 1) / CH_PHI;
    const char *gcol = reinterpret_cast<const char *>(rec + j0 * RS);
    // Folding c_i out of the pair loop needs K_ij 2^(-c_i/4096) <= 2^(-c_i/4096)
    // to stay far from overflow (with N |V| on top): whole waves whose rows
    // all have -c_i/4096 = a log2e |xc_i|^2 <= FOLD_MAX take it (the usual
    // case: particles within ~sqrt(400/a) of the mean), others the plain form.
    // The fold's u = -4096 a log2e (|x_j|^2 - 2 x_i.x_j) >= -4096 (y + 2 sqrt(400 y))
    // for y = a log2e max_j |x_j|^2: y <= 300 keeps it above -1000 x 4096, so
    // the folded form needs no clamp (nmax_bits: k_center's max |xc|^2).
    constexpr double FOLD_MAX = 400.0;
    const bool nowrap =
        nmax_bits && LOG2E * (*a_ptr) * __longlong_as_double((long long)*nmax_bits) <= 300.0;
    bool fold_ok = sgn == nullptr && nowrap; // an indefinite S can make K_ij > 1: no fold
#pragma unroll
    for (int r = 0; r < R; ++r) fold_ok = fold_ok && ci[r] >= -4096.0 * FOLD_MAX;
    const bool fold = __all(fold_ok);
    if (nch > 0) dma_to_lds<CHB>(gcol, wbuf, lane);
    constexpr bool BIAS = TABN == 8192; // biased exponent (phi_rows_pair)
    auto stream_columns = [&](auto fold_tag) {
    constexpr bool FOLD = decltype(fold_tag)::value;
    constexpr int CS = (BIAS && FOLD) ? 2 * D + 1 : 2 * D; // c_j (+ EXP_UB) slot
    for (int64_t c = 0; c < nch; ++c) {
        if (c + 1 < nch) {
            dma_to_lds<CHB>(gcol + (c + 1) * CHB, wbuf + ((c + 1) & 1) * CHB, lane);
            wait_vmcnt<CHB / 1024>();
        } else {
            wait_vmcnt<0>();
        }
        const double *cb = reinterpret_cast<const double *>(wbuf + (c & 1) * CHB);
        const int cnt = (int)min<int64_t>(CH_PHI, j1 - j0 - c * CH_PHI);
        // two register copies of the column record: the broadcast LDS reads of
        // column jj+1 are in flight while column jj is computed (the read past
        // the chunk's last column stays inside smem and is discarded)
        if constexpr (!PIPE) {
            for (int jj = 0; jj < cnt; ++jj) {
                ColRec<D> q;
                q.template load<CS>(cb + jj * RS);
                phi_rows_pair<D, R, FOLD, TABN>(q, xs, ci, acc, acc1, tab);
            }
            continue;
        }
        ColRec<D> qa, qb;
        qa.template load<CS>(cb);
        __builtin_amdgcn_s_waitcnt(0xC07F); // lgkmcnt(0): nothing pending at the loop head
        // (sched_barrier keeps the scheduler from sinking the prefetch reads
        // back down to their first use)
        // 4 columns per iteration without exit tests, then the 0..3 rest
        int jj = 0;
        for (; jj + 4 <= cnt; jj += 4) {
            qb.template load<CS>(cb + (jj + 1) * RS);
            __builtin_amdgcn_sched_barrier(0);
            phi_rows_pair<D, R, FOLD, TABN>(qa, xs, ci, acc, acc1, tab);
            __builtin_amdgcn_sched_barrier(0);
            qa.template load<CS>(cb + (jj + 2) * RS);
            __builtin_amdgcn_sched_barrier(0);
            phi_rows_pair<D, R, FOLD, TABN>(qb, xs, ci, acc, acc1, tab);
            __builtin_amdgcn_sched_barrier(0);
            qb.template load<CS>(cb + (jj + 3) * RS);
            __builtin_amdgcn_sched_barrier(0);
            phi_rows_pair<D, R, FOLD, TABN>(qa, xs, ci, acc, acc1, tab);
            __builtin_amdgcn_sched_barrier(0);
            qa.template load<CS>(cb + (jj + 4) * RS);
            __builtin_amdgcn_sched_barrier(0);
            phi_rows_pair<D, R, FOLD, TABN>(qb, xs, ci, acc, acc1, tab);
            __builtin_amdgcn_sched_barrier(0);
        }
        for (; jj < cnt; jj += 2) {
            qb.template load<CS>(cb + (jj + 1) * RS);
            __builtin_amdgcn_sched_barrier(0);
            phi_rows_pair<D, R, FOLD, TABN>(qa, xs, ci, acc, acc1, tab);
            __builtin_amdgcn_sched_barrier(0);
            if (jj + 1 >= cnt) break;
            qa.template load<CS>(cb + (jj + 2) * RS);
            __builtin_amdgcn_sched_barrier(0);
            phi_rows_pair<D, R, FOLD, TABN>(qb, xs, ci, acc, acc1, tab);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    };
    if (fold) {
        stream_columns(std::true_type{});
        // K_ij = 2^(c_i/4096) 2^((c_j + ..)/4096): the row factor, once
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const double k = __builtin_rint(ci[r]);
            const int ki = (int)k + (BIAS ? EXP_QB * EXP_TB : 0); // k in [-400 x 4096, 0]
            const double g = exp2_4096_poly(ci[r] - k) * tab_scale(tab[ki & (EXP_TB - 1)], ki);
#pragma unroll
            for (int k2 = 0; k2 < D; ++k2) acc[r][k2] *= g;
            acc1[r] *= g;
        }
    } else {
        if constexpr (BIAS)
#pragma unroll
            for (int r = 0; r < R; ++r) ci[r] += EXP_UB; // u = c_i + c_j + .. >= 0 after the clamp
        stream_columns(std::false_type{});
    }

    if constexpr (WC > 1) {
        // the WC column groups' sums, added in wave order through LDS (the
        // chunk buffers and the table are free once every wave is here), one
        // slice of 64 rows per row group at a time; coalesced partial rows
        constexpr int RB = WR * 64;  // rows of one slice
        constexpr int EL = RB * (D + 1);
        static_assert(WC * EL * 8 <= phi_rows_lds<D, NW, TABN>(), "reduction slice exceeds the LDS");
        double *red = reinterpret_cast<double *>(smem);
        __syncthreads();
#pragma unroll
        for (int r = 0; r < R; ++r) {
            double *o = red + (wc * RB + wr * 64 + lane) * (D + 1);
#pragma unroll
            for (int k = 0; k < D; ++k) o[k] = acc[r][k];
            o[D] = acc1[r];
            __syncthreads();
            for (int e = threadIdx.x; e < EL; e += NW * 64) {
                double v = red[e];
#pragma unroll
                for (int q = 1; q < WC; ++q) v += red[q * EL + e];
                const int rl = e / (D + 1), k = e - rl * (D + 1);
                const int64_t li = iblk * (WR * 64 * R) + (rl >> 6) * (64 * R) + 64 * r + (rl & 63);
                if (li < nrows) part[((int64_t)s * ldp + li) * (D + 1) + k] = v;
            }
            __syncthreads();
        }
        return;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t li = rbase + 64 * r + lane;
        if (li < nrows) {
            double *o = part + ((int64_t)s * ldp + li) * (D + 1);
#pragma unroll
            for (int k = 0; k < D; ++k) o[k] = acc[r][k];
            o[D] = acc1[r];
        }
    }
}

template <int D, int R, int NW = 4, int TABN = EXP_TB, int WC = 1>
__global__ __launch_bounds__(NW * 64) void k_phi_rows(const double *__restrict__ rec,
                                                 const double *__restrict__ a_ptr, int64_t row0,
                                                 int64_t nrows, int64_t n, int S,
                                                 double *__restrict__ part, int64_t ldp,
                                                 const double *__restrict__ sgn,
                                                 const unsigned long long *__restrict__ nmax_bits)
{
    __shared__ __attribute__((aligned(16))) char smem[phi_rows_lds<D, NW, TABN>()];
    phi_rows_body<D, R, NW, TABN, WC>(smem, blockIdx.x, rec, a_ptr, row0, nrows, n, S, part, ldp, sgn,
                                      nmax_bits);
}

// ==================================================== symmetric phi pass ==
//
// K_ij = K_ji: each unordered pair's kernel value feeds both particles.  With
// w_j = 2^(c_j/4096) = exp(-a |xc_j|^2) and E_ij = 2^(u_ij/4096),
// u_ij = 8192 a log2e xc_i.xc_j (= u_ji), K_ij = w_i w_j E_ij, so
//   S_i = sum_j E_ij W_j,   W_j = w_j [V_j, 1]   (V_j = G_j - 2a xc_j)
//   phi_i = (1/N) w_i (S_i[0..d) + 2a xc_i S_i[d])        (SVGD.hpp:453)
// and the pair (i, j) adds E_ij W_j to S_i and E_ij W_i to S_j: per
// unordered pair ONE Gram (d FMA) and ONE exp (7 VALU: the row stream's
// biased exponent and 8192-entry table, the bias riding in the Gram's first
// FMA) and 2(d+1) FMA -- instead of twice the Gram and the exp.  Valid while
// y = a log2e max|xc|^2 <= 300: then |u| <= 600 x 4096, w >= 2^-300 and
// E <= 2^600, far from over- and underflow; otherwise (symok = 0, set by
// k_prep_sym) the row stream runs instead.
//
// Work-group: SYM_NW = 8 waves (2 per SIMD); wave w holds rows
// I B + (w R + r) 64 + lane, r < R, of row block I (B = 512 R rows).  The
// column block J streams through two LDS buffers in sub-tiles of 64 records
// (global_load_lds DMA).  A sub-tile is 4 sets of 16 columns; in phase ph
// the 16-lane group g of every wave takes set (g + ph) & 3 on a skewed
// schedule: at step s lane t meets column (t + s) & 15 of the set -- its
// record is a per-lane LDS read (16 distinct records per group, an odd
// 16-byte record stride: conflict-free) -- and the set's column sums (one
// column per lane) rotate one lane per step with DPP row_ror, so BOTH sums
// stay in registers.  Per step and lane that is R unordered pairs for
// R (3d + 9) VALU, 2(d+1) + 1 DPP moves (the packet and the record address),
// R table reads and (2d+1)/2 b128 record reads -- d = 8, R = 3: 19.5 VALU
// per ordered pair-row against the row stream's 24.3.  (Round 3's version
// held R = 2 rows per lane, the unbiased exp and a 4096 table: 4.8 vs 4.7 ms.)
// After 16 steps lane t holds column (t - 1) & 15's sum over its group's
// 16 R rows; the wave's 4 groups add theirs into the wave's LDS slots
// (sCol) in phase order, and the 8 waves' are added in wave order into
// colpart (deterministic).  Row sums
// go to rowpart when the work-group's row block changes.  Diagonal tiles
// (I == J) run the row side only over the whole square (every ordered pair
// once).  k_sym_finish adds every partial of a particle in a fixed order,
// forms phi and applies the optimizer (opt_elem).
constexpr int SYM_SUB = 64; // columns per sub-tile (4 sets of 16)
constexpr int SYM_NW = 8;   // waves per work-group (2 per SIMD)
template <int D> struct SymGeom {
    // rows per lane: as many as 256 VGPRs hold at 2 waves/SIMD
    static constexpr int R = D <= 2 ? 8 : D == 3 ? 6 : D == 4 ? 5 : D == 5 ? 4 : 3;
    static constexpr int B = SYM_NW * 64 * R;            // block: a work-group's rows
    static constexpr int NSUB = B / SYM_SUB;
    static constexpr int DP = D + 1;
    // record [xc (D) | W (D+1) | pad], stride 2H doubles with H odd: a
    // group's 16 per-lane 16-byte reads hit 16 distinct 4-bank groups
    static constexpr int H = (DP % 2 == 1) ? DP : DP + 1;
    static constexpr int SRS = 2 * H;
    static constexpr int SUBB = SYM_SUB * SRS * 8;       // bytes per sub-tile (whole KiB)
    static constexpr int SCOL = SYM_NW * SYM_SUB * DP; // doubles of one column-sum buffer
    // two record buffers, the exp table, two column-sum buffers (d = 8: 154 KiB)
    static constexpr int LDS = 2 * SUBB + 8192 * 8 + 2 * SCOL * 8;
};

__device__ __forceinline__ int64_t sym_cnt(int64_t nb, int64_t I)
{
    const int64_t H = (nb - 1) / 2;
    return ((nb & 1) == 0 && I < nb / 2) ? H + 2 : H + 1;
}
__device__ __forceinline__ int64_t sym_base(int64_t nb, int64_t I)
{
    const int64_t H = (nb - 1) / 2;
    if ((nb & 1) == 0) {
        const int64_t half = nb / 2;
        return I < half ? I * (H + 2) : half * (H + 2) + (I - half) * (H + 1);
    }
    return I * (H + 1);
}

// lane t <- lane t + 1 (mod 16) within each row of 16 lanes (DPP row_ror:15)
__device__ __forceinline__ int dpp_ror15_i(int v)
{
    return __builtin_amdgcn_update_dpp(v, v, 0x12F, 0xF, 0xF, false);
}
__device__ __forceinline__ double dpp_ror15(double v)
{
    return __hiloint2double(dpp_ror15_i(__double2hiint(v)), dpp_ror15_i(__double2loint(v)));
}

// Barrier that drains only LDS operations (a __syncthreads() would also wait
// for the next sub-tile's in-flight DMA).
__device__ __forceinline__ void sym_lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// The biased 8192-entry exp table of k_phi_rows (TABN 8192) in HBM, once per
// context: k_phi_sym DMAs it into LDS instead of forming it per work-group.
__global__ void k_fill_tab8k(double *__restrict__ tab)
{
    for (int m = blockIdx.x * blockDim.x + threadIdx.x; m < 8192; m += gridDim.x * blockDim.x) {
        const double t = EXP2_TAB4096[m & (EXP_TB - 1)];
        const double tb = tab_biased(m >= EXP_TB ? 2.0 * t : t, m);
        tab[m] = __hiloint2double(__double2hiint(tb) - (EXP_QB << 20), __double2loint(tb));
    }
}
hipError_t launch_fill_tab8k(double *tab, hipStream_t stream)
{
    hipLaunchKernelGGL(k_fill_tab8k, dim3(32), dim3(256), 0, stream, tab);
    return hipGetLastError();
}

// records: srec_j = [xc_j | w_j (G_j - 2a xc_j) | w_j | 0..] (zero past n),
// w_j = exp(-a |xc_j|^2); symok = (a log2e max|xc|^2 <= 300).  When the
// symmetric form does not apply (every block sees the same flag), the row
// stream's records rec (k_prep_rec's values, rows [0, n); its padding rows
// stay zero) are written instead -- no k_prep_rec launch on the usual path.
template <int D>
__global__ void k_prep_sym(const double *__restrict__ xc, int KP, const double *__restrict__ G,
                           const double *__restrict__ nrm, const double *__restrict__ a_ptr,
                           const unsigned long long *__restrict__ nmax_bits, int64_t n, int64_t npad,
                           double *__restrict__ srec, int *__restrict__ symok, double *__restrict__ rec,
                           int RS)
{
    using Gm = SymGeom<D>;
    const double a = *a_ptr;
    const bool ok = LOG2E * a * __longlong_as_double((long long)*nmax_bits) <= 300.0;
    if (blockIdx.x == 0 && threadIdx.x == 0) *symok = ok ? 1 : 0;
    if (!ok) { // the row stream's records (k_prep_rec, same expressions)
        const int64_t tot = n * RS;
        for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
             e += (int64_t)gridDim.x * blockDim.x) {
            const int64_t j = e / RS;
            const int k = (int)(e - j * RS);
            double v = 0.0;
            if (k < D)
                v = xc[j * KP + k];
            else if (k < 2 * D)
                v = G[j * D + (k - D)] - 2.0 * a * xc[j * KP + (k - D)];
            else if (k == 2 * D)
                v = -4096.0 * a * LOG2E * nrm[j];
            else if (k == 2 * D + 1)
                v = -4096.0 * a * LOG2E * nrm[j] + EXP_UB;
            rec[e] = v;
        }
        return;
    }
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < npad;
         j += (int64_t)gridDim.x * blockDim.x) {
        double *o = srec + j * Gm::SRS;
        if (j < n) {
            const double w = exp2(-a * LOG2E * nrm[j]);
#pragma unroll
            for (int k = 0; k < D; ++k) {
                const double x = xc[j * KP + k];
                o[k] = x;
                o[D + k] = w * (G[j * D + k] - 2.0 * a * x);
            }
            o[2 * D] = w;
        } else {
#pragma unroll
            for (int k = 0; k <= 2 * D; ++k) o[k] = 0.0;
        }
#pragma unroll
        for (int k = 2 * D + 1; k < Gm::SRS; ++k) o[k] = 0.0;
    }
}

// One skew step: the lane's R rows against the column record at rj (LDS),
// whose coordinates xj the previous step already loaded (PRE: after this
// step's Gram, the next record's coordinates rn are loaded into xj -- their
// LDS latency then hides behind this step's exp and accumulation instead of
// stalling the next step's Gram; xj's registers are free after the Gram).
// SYMM: also the column side into cacc; ROT: then rotate cacc one lane.
#ifndef SVGD_SYM_PRE
#define SVGD_SYM_PRE 1
#endif
template <int D>
__device__ __forceinline__ void sym_load_x(const double *rj, double (&xj)[D + (D & 1)])
{
    // 16-byte LDS reads of the lane's record (ds_read_b128: 16-lane groups,
    // the odd 16-byte record stride conflict-free).  The records are 16-byte
    // aligned (SRS even, whole-KiB buffers), but without the hint the
    // compiler emits ds_read2_b64 pairs, whose 32-bank rule puts records r
    // and r + 8 on the same banks: every record read 2-way conflicted.
    const double2 *r2 = reinterpret_cast<const double2 *>(__builtin_assume_aligned(rj, 16));
#pragma unroll
    for (int q = 0; q < (D + 1) / 2; ++q) {
        const double2 t = r2[q];
        xj[2 * q] = t.x;
        xj[2 * q + 1] = t.y;
    }
}
template <int D, int R, bool SYMM, bool ROT, bool PRE>
__device__ __forceinline__ void sym_step(const double *rj, const double *rn, double (&xj)[D + (D & 1)],
                                         const double (&xs)[R][D], const double (&wr)[R][D + 1],
                                         double (&acc)[R][D + 1], double (&cacc)[D + 1], const double *tab)
{
    constexpr int DP = D + 1;
    __builtin_amdgcn_sched_barrier(0);
    double u[R];
    const double2 *r2 = reinterpret_cast<const double2 *>(__builtin_assume_aligned(rj, 16));
#pragma unroll
    for (int r = 0; r < R; ++r) u[r] = fma(xs[r][0], xj[0], EXP_UB); // biased: u >= 0
#pragma unroll
    for (int k = 1; k < D; ++k)
#pragma unroll
        for (int r = 0; r < R; ++r) u[r] = fma(xs[r][k], xj[k], u[r]);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PRE) sym_load_x<D>(rn, xj);
    double wj[DP + 1];
    if constexpr (D % 2 == 0) { // W at a 16-byte boundary: (D + 2) / 2 reads
#pragma unroll
        for (int q = 0; q < (DP + 1) / 2; ++q) {
            const double2 t = r2[D / 2 + q];
            wj[2 * q] = t.x;
            wj[2 * q + 1] = t.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < DP; ++k) wj[k] = rj[D + k];
    }
    double f[R], T[R], E[R];
    int ki[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        f[r] = __builtin_amdgcn_fract(u[r]); // u >= 0: u - floor(u)
        ki[r] = (int)u[r];                    // = floor(u)
        T[r] = *reinterpret_cast<const double *>(reinterpret_cast<const char *>(tab) + tab8k_offset(ki[r]));
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < R; ++r) E[r] = exp2_4096_poly01(f[r]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < R; ++r) E[r] = E[r] * tab_scale(T[r], ki[r]);
#pragma unroll
    for (int k = 0; k < DP; ++k)
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r][k] = fma(E[r], wj[k], acc[r][k]);
    if constexpr (SYMM) {
#pragma unroll
        for (int k = 0; k < DP; ++k) {
            double c = cacc[k];
#pragma unroll
            for (int r = 0; r < R; ++r) c = fma(E[r], wr[r][k], c);
            cacc[k] = ROT ? dpp_ror15(c) : c;
        }
    }
    __builtin_amdgcn_sched_barrier(0);
}

// The 4 phases of one sub-tile (buffer cb) for this wave: group grp takes
// set (grp + ph) & 3 in phase ph, 16 skew steps each; SYMM: the set's column
// sums go to this wave's sCol slots.
template <int D, bool SYMM>
__device__ __forceinline__ void sym_phases(const char *cb, int grp, int tl, int w,
                                           const double (&xs)[SymGeom<D>::R][D],
                                           const double (&wr)[SymGeom<D>::R][D + 1],
                                           double (&acc)[SymGeom<D>::R][D + 1], double *sCol,
                                           const double *tab)
{
    using Gm = SymGeom<D>;
    constexpr int R = Gm::R, SRS = Gm::SRS, DP = Gm::DP;
#pragma unroll 1
    for (int ph = 0; ph < 4; ++ph) {
        const int set = (grp + ph) & 3;
        // this lane's record at step s: column (tl + s) & 15 of the set; the
        // byte offset rotates with the column packet
        int roff = (set * 16 + tl) * SRS * 8;
        double cacc[DP];
#pragma unroll
        for (int k = 0; k < DP; ++k) cacc[k] = 0.0;
        // 16 steps straight-line: the last one leaves the packet in place
        double xj[D + (D & 1)];
        sym_load_x<D>(reinterpret_cast<const double *>(cb + roff), xj);
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            if (s < 15) {
                const int rnext = dpp_ror15_i(roff);
                if constexpr (SVGD_SYM_PRE) {
                    sym_step<D, R, SYMM, true, true>(reinterpret_cast<const double *>(cb + roff),
                                                     reinterpret_cast<const double *>(cb + rnext), xj, xs, wr,
                                                     acc, cacc, tab);
                } else {
                    sym_step<D, R, SYMM, true, false>(reinterpret_cast<const double *>(cb + roff), nullptr, xj,
                                                      xs, wr, acc, cacc, tab);
                    sym_load_x<D>(reinterpret_cast<const double *>(cb + rnext), xj);
                }
                roff = rnext;
            } else {
                sym_step<D, R, SYMM, false, false>(reinterpret_cast<const double *>(cb + roff), nullptr, xj, xs,
                                                   wr, acc, cacc, tab);
            }
        }
        if constexpr (SYMM) {
            // lane t holds column (t - 1) & 15's sum over this group's rows;
            // the wave's 4 groups (different rows) visit every set once, in
            // phase order, and add into the wave's zeroed slots (in order
            // within the wave: deterministic; a branch on the phase here
            // would let the compiler peel the 16-step body and spill)
            double *sc = sCol + (w * SYM_SUB + set * 16 + ((tl + 15) & 15)) * DP;
#pragma unroll
            for (int k = 0; k < DP; ++k) sc[k] += cacc[k];
        }
    }
}

// The row stream's hand-over (symok = 0): its 8-wave work-groups (grid of
// them: row groups of 256 rows x S column splits) over the rank's rows,
// partials into part (S x ldp x (d+1)).
struct SymRows {
    const double *rec;
    int64_t row0, nrows, n;
    int S;
    int64_t grid;
    double *part;
    int64_t ldp;
    const unsigned long long *nmax;
};

template <int D>
__global__ __launch_bounds__(SYM_NW * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_phi_sym(
    const double *__restrict__ srec, const double *__restrict__ a_ptr, int64_t nb, int64_t U0, int64_t U1,
    const int *__restrict__ symok, double *__restrict__ rowpart, const int *__restrict__ blkg,
    const int *__restrict__ rbase, double *__restrict__ colpart, int64_t SM, const int *__restrict__ wst,
    int qlast, const double *__restrict__ tab8k, SymRows fr)
{
    using Gm = SymGeom<D>;
    constexpr int R = Gm::R, B = Gm::B, NSUB = Gm::NSUB, SRS = Gm::SRS, DP = Gm::DP,
                  SUBB = Gm::SUBB, NP = SUBB / 1024, NT = SYM_NW * 64;
    __shared__ __attribute__((aligned(16))) char smem[Gm::LDS];
    if (!*symok) {
        // uniform: the symmetric form would leave its exponent range, the
        // row stream takes the step in this launch (its work-groups looped
        // over this grid; the same code, LDS and partials as k_phi_rows)
        static_assert(T8K_NW == SYM_NW && phi_rows_lds<D, T8K_NW, 8192>() <= Gm::LDS,
                      "the row stream's work-group must fit the symmetric pass's");
        for (int64_t b = blockIdx.x; b < fr.grid; b += gridDim.x) {
            phi_rows_body<D, 4, T8K_NW, 8192, T8K_WC>(smem, b, fr.rec, a_ptr, fr.row0, fr.nrows, fr.n, fr.S,
                                                      fr.part, fr.ldp, nullptr, fr.nmax);
            __syncthreads(); // (the next work-group's table fill reuses the LDS)
        }
        return;
    }
    double *tab = reinterpret_cast<double *>(smem + 2 * SUBB);
    double *sCol = tab + 8192; // [2][SYM_NW][SYM_SUB][DP]: sub-tile u's column sums in buffer u & 1
    constexpr int SCOL = Gm::SCOL;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = lane >> 4, tl = lane & 15;

    const double alpha = 8192.0 * LOG2E * (*a_ptr);
    // this work-group's contiguous run of the rank's units [U0, U1)
    const int64_t Gn = gridDim.x, V = U1 - U0;
    const int64_t u0 = U0 + V * (int64_t)blockIdx.x / Gn, u1 = U0 + V * ((int64_t)blockIdx.x + 1) / Gn;
    // (tile, sub-tile) cursor: the plan's tile t = (I, J), J = I + slot mod nb
    // (plan.cpp), nq sub-tiles in it (qlast for the last column block: its
    // padding-only sub-tiles are no units); the run's first unit from the
    // host's table wst, then advanced incrementally (no 64-bit divisions)
    struct Cur {
        int64_t t, I, J, slot, cnt;
        int q, nq;
    };
    auto cur_start = [&]() {
        Cur c;
        c.t = wst[2 * blockIdx.x];
        c.q = wst[2 * blockIdx.x + 1];
        tile_coords(nb, c.t, &c.I, &c.J);
        c.slot = c.J >= c.I ? c.J - c.I : c.J + nb - c.I;
        c.cnt = sym_cnt(nb, c.I);
        c.nq = c.J == nb - 1 ? qlast : NSUB;
        return c;
    };
    auto cur_next = [&](Cur &c) {
        if (++c.q < c.nq) return;
        c.q = 0;
        ++c.t;
        if (++c.slot == c.cnt) {
            ++c.I;
            c.slot = 0;
            c.cnt = sym_cnt(nb, c.I);
        }
        c.J = c.I + c.slot >= nb ? c.I + c.slot - nb : c.I + c.slot;
        c.nq = c.J == nb - 1 ? qlast : NSUB;
    };
    auto issue = [&](const Cur &c, int buf) {
        const char *src =
            reinterpret_cast<const char *>(srec + (c.J * B + (int64_t)c.q * SYM_SUB) * SRS);
        char *dst = smem + buf * SUBB;
        for (int p = w; p < NP; p += SYM_NW)
            __builtin_amdgcn_global_load_lds((gbl_void *)(src + p * 1024 + lane * 16),
                                             (lds_void *)(dst + p * 1024), 16, 0, 0);
    };

    double xs[R][D], wr[R][DP], acc[R][DP];
    int64_t curI = -1;
    // row sums of block curI -> rowpart record rbase[curI] + (this group -
    // the first group visiting curI): each row block's records contiguous,
    // in work-group order (the finish reads them as one run)
#define SYM_FLUSH_ROWS()                                                                        \
    do {                                                                                        \
        double *o_ = rowpart + ((int64_t)rbase[curI] + ((int)blockIdx.x - blkg[2 * curI])) * B * DP; \
        _Pragma("unroll") for (int r = 0; r < R; ++r) {                                         \
            const int lr = (w * R + r) * 64 + lane;                                             \
            _Pragma("unroll") for (int k = 0; k < DP; ++k) o_[lr * DP + k] = acc[r][k];         \
        }                                                                                       \
    } while (0)

    if (u0 >= u1) return;
    // Prologue, its memory latencies overlapped: the DMA of the biased
    // 8192-entry exp table (the row stream's, k_phi_rows TABN 8192, filled
    // once per context into tab8k: 64 pieces of 1 KiB) and of the first
    // sub-tile, then the first row block's registers, then the column-sum
    // buffers zeroed; the loop's first barrier (after vmcnt(0)) covers all.
    for (int p = w; p < 64; p += SYM_NW)
        __builtin_amdgcn_global_load_lds((gbl_void *)(reinterpret_cast<const char *>(tab8k) + p * 1024 + lane * 16),
                                         (lds_void *)(reinterpret_cast<char *>(tab) + p * 1024), 16, 0, 0);
    // One barrier per sub-tile: the column sums of sub-tile u go to buffer
    // u & 1 and are added into colpart during sub-tile u + 1 (after its
    // barrier, when every wave is past sub-tile u), and the DMA of sub-tile
    // u + 1 is issued right after that barrier (every wave is then done with
    // the record buffer it refills).  The barrier of sub-tile u + 1 also
    // orders the zeroing of a column buffer before its next use.
    // the 8 waves' column sums of a sub-tile added in wave order into
    // colpart[J][slot] (off the diagonal: a diagonal tile's are dropped), the
    // buffer zeroed; colpart by (column block, slot), so a particle's column
    // terms are one run (the finish); entries no unit of this rank writes
    // stay zero from the allocation
    auto col_out = [&](double *scw, int64_t Jp, int64_t slotp, int qp, bool diagp) {
        double *o = colpart + ((Jp * SM + slotp) * B + (int64_t)qp * SYM_SUB) * DP;
        for (int e = tid; e < SYM_SUB * DP; e += NT) {
            double v = scw[e];
            scw[e] = 0.0;
#pragma unroll
            for (int ww = 1; ww < SYM_NW; ++ww) {
                v += scw[ww * SYM_SUB * DP + e];
                scw[ww * SYM_SUB * DP + e] = 0.0;
            }
            if (!diagp) o[e] = v;
        }
    };
    Cur cu = cur_start(), cn = cu;
    issue(cu, 0);
    curI = cu.I;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const double *ri = srec + (curI * B + (w * R + r) * 64 + lane) * SRS;
#pragma unroll
        for (int k = 0; k < D; ++k) xs[r][k] = alpha * ri[k];
#pragma unroll
        for (int k = 0; k < DP; ++k) {
            wr[r][k] = ri[D + k];
            acc[r][k] = 0.0;
        }
    }
    for (int e = tid; e < 2 * SCOL; e += NT) sCol[e] = 0.0;
    int64_t pJ = 0, pSlot = 0;
    int pQ = 0;
    bool pDiag = true, have_prev = false;
    for (int64_t u = u0; u < u1; ++u) {
        const int buf = (int)((u - u0) & 1);
        wait_vmcnt<0>();   // this wave's pieces of sub-tile u (the only DMA in flight)
        sym_lds_barrier(); // every wave's pieces are in LDS; every wave is past sub-tile u - 1
        if (u + 1 < u1) {
            cur_next(cn);
            issue(cn, buf ^ 1);
        }
        if (have_prev) col_out(sCol + (buf ^ 1) * SCOL, pJ, pSlot, pQ, pDiag);
        const int64_t I = cu.I, J = cu.J, slot = cu.slot;
        const int q = cu.q;
        cur_next(cu);
        pJ = J;
        pSlot = slot;
        pQ = q;
        pDiag = I == J;
        have_prev = true;
        if (I != curI) {
            if (curI >= 0) SYM_FLUSH_ROWS();
            curI = I;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const double *ri = srec + (I * B + (w * R + r) * 64 + lane) * SRS;
#pragma unroll
                for (int k = 0; k < D; ++k) xs[r][k] = alpha * ri[k];
#pragma unroll
                for (int k = 0; k < DP; ++k) {
                    wr[r][k] = ri[D + k];
                    acc[r][k] = 0.0;
                }
            }
            wait_vmcnt<0>(); // (rare: once per row block) also drains the next sub-tile's DMA
        }
        const char *cb = smem + buf * SUBB;
        // one code path for both tile kinds (two would double the live
        // register ranges: the allocator spilled); a diagonal tile's column
        // sums are computed and dropped -- its row side already holds every
        // ordered pair of the square (~2 % of the tiles)
        sym_phases<D, true>(cb, grp, tl, w, xs, wr, acc, sCol + buf * SCOL, tab);
    }
    sym_lds_barrier(); // every wave's column sums of the last sub-tile are in LDS
    col_out(sCol + ((u1 - 1 - u0) & 1) * SCOL, pJ, pSlot, pQ, pDiag);
    if (curI >= 0) SYM_FLUSH_ROWS();
#undef SYM_FLUSH_ROWS
}

// The row stream's step when the symmetric form does not apply (symok = 0):
// its partials (launch_phi_rows without its reduce) summed per element in
// split order and phi_i = (S_i[0..d) + 2a xc_i S_i[d]) / N -- k_phi_reduce's
// arithmetic in the symmetric finish's block geometry (256 / (d+1) rows).
struct SymFallback {
    const double *part; // S x ldp x (d+1)
    int S;
    int64_t ldp;
    const double *rec; // the row records (xc in slots 0..d)
    int RS;
};
template <int D>
__device__ __forceinline__ double sym_fb_sum(const SymFallback &fb, int64_t rb, int e)
{
    constexpr int DP = D + 1;
    const double *p = fb.part + rb * DP + e;
    const int64_t st = fb.ldp * DP;
    double acc = 0.0;
    for (int s0 = 0; s0 < fb.S; s0 += 16) { // 16 splits' loads in flight, added in s order
        double v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = s0 + q < fb.S ? p[(s0 + q) * st] : 0.0;
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if (s0 + q < fb.S) acc += v[q];
    }
    return acc;
}
template <int D>
__device__ __forceinline__ void sym_fb_phi(const SymFallback &fb, const double *sm, int64_t rb, int rows,
                                           int64_t row0, double inv_n, double a, double *phi,
                                           const OptArgs &opt, int do_opt)
{
    constexpr int DP = D + 1;
    for (int o = threadIdx.x; o < rows * D; o += blockDim.x) {
        const int r = o / D, k = o - r * D;
        const int64_t li = rb + r;
        const double w = 2.0 * a * fb.rec[(row0 + li) * fb.RS + k];
        const double ph = inv_n * (sm[r * DP + k] + w * sm[r * DP + D]);
        phi[li * D + k] = ph;
        if (do_opt) opt_elem(opt, li * D + k, ph);
    }
}
// phi_p = (1/N) w_p (S_p[0..d) + 2a xc_p S_p[d]) for this rank's rows, S_p =
// every row and column partial of p in a fixed order, then the optimizer.
// A block owns 256 / (d+1) particles, one thread per (particle, component).
// The partials are those of the units [U0, U1) (this rank's) run by G
// work-groups.  contrib (P > 1): instead of phi, S_p from this rank's units
// alone -> contrib[p * DP + k] for the particles those units touch (rows
// [row0, row0 + nrows) a cyclic run, p taken mod nwrap), the send buffer of
// the point-to-point exchange; k_sym_apply then forms phi.
template <int D>
__global__ __launch_bounds__(256) void k_sym_finish(const double *__restrict__ rowpart,
                                                    const double *__restrict__ colpart,
                                                    const double *__restrict__ srec,
                                                    const double *__restrict__ a_ptr, int64_t nb,
                                                    int64_t SM, int64_t Ia, int64_t Ib,
                                                    const int *__restrict__ blkg,
                                                    const int *__restrict__ rbase,
                                                    const int *__restrict__ symok, int64_t row0,
                                                    int64_t nrows, double inv_n, double *__restrict__ phi,
                                                    OptArgs opt, int do_opt, double *__restrict__ contrib,
                                                    int64_t nwrap, SymFallback fb)
{
    using Gm = SymGeom<D>;
    constexpr int B = Gm::B, SRS = Gm::SRS, DP = Gm::DP, RB = 256 / DP;
    const bool ok = *symok;
    if (!ok && contrib) return; // (k_sym_apply takes the row stream's step)
    __shared__ double sm[256];
    const int64_t rb = (int64_t)blockIdx.x * RB;
    const int rows = (int)min<int64_t>(RB, nrows - rb);
    if (rows <= 0) return;
    const int e = threadIdx.x;
    if (!ok) { // the row stream took the step: its partials, then its phi form
        if (e < rows * DP) sm[e] = sym_fb_sum<D>(fb, rb, e);
        __syncthreads();
        sym_fb_phi<D>(fb, sm, rb, rows, row0, inv_n, *a_ptr, phi, opt, do_opt);
        return;
    }
    if (e < rows * DP) {
        const int pl_ = e / DP, k = e - pl_ * DP;
        int64_t p = row0 + rb + pl_;
        if (nwrap && p >= nwrap) p -= nwrap; // (contrib: a cyclic run of particles)
        const int64_t P = p / B, pl = p - P * B;
        double acc = 0.0;
        // row role: the row sums of the work-groups that visited row block P,
        // one contiguous run (k_phi_sym's rowpart layout), in work-group order
        {
            const int cnt = blkg[2 * P + 1] - blkg[2 * P] + 1; // <= 0: none
            const double *rp = rowpart + ((int64_t)rbase[P] * B + pl) * DP + k;
            for (int i0 = 0; i0 < cnt; i0 += 16) {
                double v[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) v[u] = i0 + u < cnt ? rp[(int64_t)(i0 + u) * B * DP] : 0.0;
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (i0 + u < cnt) acc += v[u];
            }
        }
        // column role: colpart[P][slot], slots 1 .. SM-1 in order (entries no
        // unit of this rank wrote are zero); a rank whose units span the row
        // blocks Ia .. Ib only (P > 1) reads the slots P - I of those, fewer
        // -- 16 loads in flight
        const double *cp = colpart + ((P * SM) * B + pl) * DP + k;
        const int64_t cs = (int64_t)B * DP;
        if (Ib - Ia + 1 >= SM - 1) {
            for (int64_t s0 = 1; s0 < SM; s0 += 16) {
                double v[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) v[u] = s0 + u < SM ? cp[(s0 + u) * cs] : 0.0;
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (s0 + u < SM) acc += v[u];
            }
        } else {
            for (int64_t i0 = Ia; i0 <= Ib; i0 += 16) {
                double v[16];
                bool okv[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    int64_t sl = P - (i0 + u);
                    if (sl < 0) sl += nb;
                    okv[u] = i0 + u <= Ib && sl >= 1 && sl < SM;
                    v[u] = okv[u] ? cp[sl * cs] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (okv[u]) acc += v[u];
            }
        }
        if (contrib) {
            contrib[p * DP + k] = acc;
            return;
        }
        sm[e] = acc;
    }
    if (contrib) return;
    __syncthreads();
    const double two_a = 2.0 * (*a_ptr);
    for (int o = threadIdx.x; o < rows * D; o += blockDim.x) {
        const int r = o / D, k = o - r * D;
        const int64_t li = rb + r, p = row0 + li;
        const double *rec = srec + p * SRS;
        const double ph = inv_n * (rec[2 * D] * (sm[r * DP + k] + two_a * rec[k] * sm[r * DP + D]));
        phi[li * D + k] = ph;
        if (do_opt) opt_elem(opt, li * D + k, ph);
    }
}

// P > 1: phi and the optimizer for this rank's rows from the sums of every
// rank's contributions, added in rank order: this rank's own (own, nrows x
// DP) and the pieces received from the others (xtab: per rank q its rows
// [t0, t1) at recv + off rows, t1 <= t0: none; q == rank: own) -- or from
// the row stream's partials when it took the step (symok = 0); the finish's
// block geometry.
template <int D>
__global__ __launch_bounds__(256) void k_sym_apply(const double *__restrict__ own, const double *__restrict__ recv,
                                                   const int64_t *__restrict__ xtab, int world, int rank,
                                                   const double *__restrict__ srec,
                                                   const double *__restrict__ a_ptr,
                                                   const int *__restrict__ symok, int64_t row0, int64_t nrows,
                                                   double inv_n, double *__restrict__ phi, OptArgs opt,
                                                   int do_opt, SymFallback fb)
{
    using Gm = SymGeom<D>;
    constexpr int SRS = Gm::SRS, DP = Gm::DP, RB = 256 / DP;
    __shared__ double sm[256];
    const bool ok = *symok;
    const int64_t rb = (int64_t)blockIdx.x * RB;
    const int rows = (int)min<int64_t>(RB, nrows - rb);
    if (rows <= 0) return;
    const int e = threadIdx.x;
    if (e < rows * DP) {
        if (ok) {
            const int pl = e / DP, k = e - pl * DP;
            const int64_t p = row0 + rb + pl;
            double v = 0.0;
            for (int q = 0; q < world; ++q) {
                if (q == rank) {
                    v += own[rb * DP + e];
                } else {
                    const int64_t t0 = xtab[3 * q], t1 = xtab[3 * q + 1];
                    if (p >= t0 && p < t1) v += recv[(xtab[3 * q + 2] + (p - t0)) * DP + k];
                }
            }
            sm[e] = v;
        } else {
            sm[e] = sym_fb_sum<D>(fb, rb, e);
        }
    }
    __syncthreads();
    if (!ok) {
        sym_fb_phi<D>(fb, sm, rb, rows, row0, inv_n, *a_ptr, phi, opt, do_opt);
        return;
    }
    const double two_a = 2.0 * (*a_ptr);
    for (int o = threadIdx.x; o < rows * D; o += blockDim.x) {
        const int r = o / D, k = o - r * D;
        const int64_t li = rb + r;
        const double *rec = srec + (row0 + li) * SRS;
        const double ph = inv_n * (rec[2 * D] * (sm[r * DP + k] + two_a * rec[k] * sm[r * DP + D]));
        phi[li * D + k] = ph;
        if (do_opt) opt_elem(opt, li * D + k, ph);
    }
}

// ------------------------------------------- fp32 tile phi, streamed (F32) --
//
// k_phi<float>'s arithmetic (Gram on v_mfma_f32_16x16x4f32, P = 2^t by
// v_exp_f32, acc += P V on the MFMA), restructured for the fp32 MFMA rate:
// the column tiles (32 particles) stream through two LDS buffers by
// global_load_lds DMA -- the next tile lands while the current one is
// computed, one barrier per tile -- from operand-ordered copies made once per
// step (k_swz_f32), so every LDS read is a conflict-free 16-byte read of 64
// consecutive lanes:
//   XS[t][js][u][lane][e]  = x[32t + 16js + lane%16][16u + 4(lane/16) + e]
//                           (the Gram A operand of MFMA step 4u+e, kslot order)
//   VS[t][js][cb][lane][r] = V[32t + 16js + 4(lane/16) + r][16cb + lane%16]
//                           (the P.V B operand of step r), plane NCB: c_j
// Rows (B operand of the Gram) come from the row-major fp32 copy in the same
// kslot order.  Wave w owns rows 16w..16w+15 of the block's 64.
constexpr int TBJ = 32; // columns per streamed tile

__global__ void k_swz_f32(const double *__restrict__ x, int KP, const double *__restrict__ V,
                          int VW, const double *__restrict__ cvec, int64_t ntiles,
                          float *__restrict__ XS, float *__restrict__ VS)
{
    const int KU = KP / 16, NCB = VW / 16;
    const int64_t nx = ntiles * TBJ * KP, nv = ntiles * 2 * (NCB + 1) * 256;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nx + nv;
         e += (int64_t)gridDim.x * blockDim.x) {
        if (e < nx) {
            const int q4 = (int)(e & 3), lane = (int)((e >> 2) & 63);
            int64_t r = e >> 8;
            const int u = (int)(r % KU);
            r /= KU;
            const int js = (int)(r & 1);
            const int64_t t = r >> 1;
            const int64_t j = t * TBJ + 16 * js + (lane & 15);
            XS[e] = (float)x[j * KP + 16 * u + 4 * (lane >> 4) + q4];
        } else {
            const int64_t f = e - nx;
            const int rr = (int)(f & 3), lane = (int)((f >> 2) & 63);
            int64_t r = f >> 8;
            const int cb = (int)(r % (NCB + 1));
            r /= (NCB + 1);
            const int js = (int)(r & 1);
            const int64_t t = r >> 1;
            const int64_t j = t * TBJ + 16 * js + 4 * (lane >> 4) + rr;
            VS[f] = cb < NCB ? (float)V[j * VW + 16 * cb + (lane & 15)] : (float)cvec[j];
        }
    }
}

template <int KP, int NCB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_phi_f32s(
    const float *__restrict__ XS, const float *__restrict__ VS, const float *__restrict__ xrow,
    const float *__restrict__ crow, const double *__restrict__ a_ptr, int64_t row0, int64_t nrows,
    int64_t ntiles, int d, double inv_n, const double *__restrict__ wv,
    const double *__restrict__ xc, int xc_stride, double *__restrict__ phi, OptArgs opt, int do_opt)
{
    constexpr int KK = KP / 4, KU = KP / 16;
    constexpr int VW = 16 * NCB;
    constexpr int PX = 2 * KU, PV = 2 * (NCB + 1); // 1 KiB pieces per tile
    constexpr int BUF = (PX + PV) * 256;            // floats per LDS buffer
    __shared__ __attribute__((aligned(16))) float sbuf[2 * BUF];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lo = lane & 15, hi = lane >> 4;
    const double a = *a_ptr;
    const float alpha = (float)(2.0 * a * LOG2E);

    const int64_t ibase = row0 + (int64_t)blockIdx.x * 64 + w * 16;
    float bI[KK];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) bI[kk] = xrow[(ibase + lo) * KP + kslot<float, KP>(kk, hi)];
    const float ci = crow[ibase + lo];

    f4_t acc[NCB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) acc[cb] = f4_t{0.0f, 0.0f, 0.0f, 0.0f};

    // this wave's share of tile t's DMA pieces into buffer b
    auto issue = [&](int64_t t, int b) {
        const char *gx = reinterpret_cast<const char *>(XS + t * (PX * 256));
        const char *gv = reinterpret_cast<const char *>(VS + t * (PV * 256));
        char *lb = reinterpret_cast<char *>(sbuf + b * BUF);
#pragma unroll
        for (int p = w; p < PX + PV; p += 4) {
            const char *g = p < PX ? gx + p * 1024 : gv + (p - PX) * 1024;
            __builtin_amdgcn_global_load_lds((gbl_void *)(g + lane * 16), (lds_void *)(lb + p * 1024), 16, 0, 0);
        }
    };
    if (ntiles > 0) issue(0, 0);
    for (int64_t t = 0; t < ntiles; ++t) {
        const int b = (int)(t & 1);
        wait_vmcnt<0>();  // this wave's pieces of tile t
        __syncthreads(); // everyone's pieces; everyone is done with buffer b ^ 1
        if (t + 1 < ntiles) issue(t + 1, b ^ 1);
        const float *lx = sbuf + b * BUF, *lv = lx + PX * 256;
#pragma unroll
        for (int js = 0; js < 2; ++js) {
            float A[KK];
#pragma unroll
            for (int u = 0; u < KU; ++u) {
                const f4_t q = *reinterpret_cast<const f4_t *>(lx + (js * KU + u) * 256 + lane * 4);
#pragma unroll
                for (int e = 0; e < 4; ++e) A[4 * u + e] = q[e];
            }
            f4_t dot = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int kk = 0; kk < KK; ++kk)
                dot = __builtin_amdgcn_mfma_f32_16x16x4f32(A[kk], bI[kk], dot, 0, 0, 0);
            const f4_t cj = *reinterpret_cast<const f4_t *>(lv + (js * (NCB + 1) + NCB) * 256 + lane * 4);
            f4_t vv[NCB];
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb)
                vv[cb] = *reinterpret_cast<const f4_t *>(lv + (js * (NCB + 1) + cb) * 256 + lane * 4);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float p = exp2_nonpos(fmaf(alpha, dot[r], ci + cj[r]));
#pragma unroll
                for (int cb = 0; cb < NCB; ++cb)
                    acc[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(p, vv[cb][r], acc[cb], 0, 0, 0);
            }
        }
    }

    // epilogue (fp64), through LDS (the tile buffers are free after the barrier)
    __syncthreads();
    float *sAcc = sbuf + w * 16 * (VW + 1);
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int q = 0; q < 4; ++q) sAcc[(4 * hi + q) * (VW + 1) + cb * 16 + lo] = acc[cb][q];
    __syncthreads();
    const double two_a = 2.0 * a;
    for (int e = lane; e < 16 * d; e += 64) {
        const int il = e / d, c = e - il * d;
        const int64_t i = ibase + il;
        if (i - row0 < nrows) {
            const double s1 = (double)sAcc[il * (VW + 1) + d];
            const double wgt = wv ? wv[i * d + c] : two_a * xc[i * xc_stride + c];
            const double ph = inv_n * ((double)sAcc[il * (VW + 1) + c] + wgt * s1);
            phi[(i - row0) * d + c] = ph;
            if (do_opt) opt_elem(opt, (i - row0) * d + c, ph);
        }
    }
}

// ------------------------- fp32 tile phi on the bf16 matrix cores (F32, B3) --
//
// The F32 path's arithmetic at the bf16 MFMA rate (16x the f32 MFMA's on
// gfx950): every fp32 operand is split exactly into three bf16 parts,
// x = h + m + l (8 + 8 + 8 significant bits), and each fp32 product a.b is
// formed from the six part products that reach 2^-24 of it -- hh, hm, mh,
// hl, lh, mm (the dropped ml, lm, ll are < 2^-23 |a b|): the Gram and the
// P.V contraction keep fp32-level accuracy, both on v_mfma_f32_16x16x32_bf16
// (products exact, fp32 accumulation).  Per 16 x 16 pair block: 6 KP/32
// Gram MFMAs and (per 32 columns) 6 NCB P.V MFMAs of 16 cycles instead of
// KP/4 + 4 NCB f32 MFMAs of 32.  P = 2^t by v_exp_f32 as k_phi_f32s; P's three
// parts are formed in registers, P already being the P.V A operand in the
// 16x16x32 lane map (lane l: row l%16, k = 8(l/16) + e).
// Operand-ordered parts, once per step (k_swz_b3), per 32-column tile t, in
// 1 KiB pieces of 64 lanes x 16 bytes:
//   XB[t][js][db][part][lane][e] = part of x[32t + 16js + lane%16][32db + 8(lane/16) + e]
//   VB[t][cb][part][lane][e]     = part of V[32t + 16(e/4) + 4(lane/16) + e%4][16cb + lane%16]
//   CB[t][js][lane][r]           = c_j (fp32), j = 32t + 16js + 4(lane/16) + r
// Rows (the Gram's B operand) come from XB of the row's own tile: the same
// lane map.
// Truncating form (exact as well: h = the top 16 bits of x, x - h exact with
// at most 16 significant bits, and so on; |m| < 2^-7 |x|, |l| < 2^-15 |x|):
// the high halves of two floats packed by one v_perm, the residual by a mask
// and a packed subtract -- no conversion instructions
__device__ __forceinline__ uint32_t b3_trunc_pair(float &x0, float &x1)
{
    const uint32_t u0 = __float_as_uint(x0), u1 = __float_as_uint(x1);
    const uint32_t w = __builtin_amdgcn_perm(u1, u0, 0x07060302u); // hi16(x1) << 16 | hi16(x0)
    typedef float f2v __attribute__((ext_vector_type(2)));
    const f2v r = f2v{x0, x1} - f2v{__uint_as_float(u0 & 0xffff0000u), __uint_as_float(u1 & 0xffff0000u)};
    x0 = r[0];
    x1 = r[1];
    return w;
}
#ifndef SVGD_B3_TRUNC
#define SVGD_B3_TRUNC 1
#endif

__device__ __forceinline__ uint32_t b3_split_pair(float &x0, float &x1)
{
    // bf16(x0) | bf16(x1) << 16 (round to nearest even), and the residuals
    // x - bf16(x) back in x0, x1 (exact in fp32)
    uint32_t w;
    asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(w) : "v"(x0), "v"(x1));
    x0 -= __uint_as_float(w << 16);
    x1 -= __uint_as_float(w & 0xffff0000u);
    return w;
}

template <int KP>
__global__ void k_swz_b3(const double *__restrict__ x, const double *__restrict__ V, int VW,
                         const double *__restrict__ cvec, int64_t n, int64_t ntiles,
                         uint32_t *__restrict__ B3)
{
    // one thread per (piece, lane) pair of elements: 4 dwords (8 bf16) of one
    // part, the three parts of one (row, 8-k) slice formed together
    constexpr int NDB = KP / 32;
    const int NCB = VW / 16;
    const int PT = 6 * NDB + 3 * NCB + 2; // pieces per tile
    const int64_t nslices = ntiles * (2 * NDB + NCB) * 64; // (lane, slice) items of XB and VB
    const int64_t ncb = ntiles * 2 * 64;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nslices + ncb;
         e += (int64_t)gridDim.x * blockDim.x) {
        if (e < nslices) {
            const int lane = (int)(e & 63);
            int64_t r = e >> 6;
            const int sl = (int)(r % (2 * NDB + NCB));
            const int64_t t = r / (2 * NDB + NCB);
            const int lo = lane & 15, hi = lane >> 4;
            float v[8];
            int piece0;
            if (sl < 2 * NDB) { // XB slice (js, db)
                const int js = sl / NDB, db = sl - js * NDB;
                const int64_t j = t * 32 + 16 * js + lo;
#pragma unroll
                for (int q = 0; q < 8; ++q) v[q] = (float)x[j * KP + 32 * db + 8 * hi + q];
                piece0 = (js * NDB + db) * 3;
            } else { // VB slice cb
                const int cb = sl - 2 * NDB;
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int64_t j = t * 32 + 16 * (q >> 2) + 4 * hi + (q & 3);
                    v[q] = (float)V[j * VW + 16 * cb + lo];
                }
                piece0 = 6 * NDB + 3 * cb;
            }
            uint32_t *o = B3 + (t * PT + piece0) * 256 + lane * 4;
#pragma unroll
            for (int part = 0; part < 3; ++part)
#pragma unroll
                for (int q = 0; q < 4; ++q) o[part * 256 + q] = b3_split_pair(v[2 * q], v[2 * q + 1]);
        } else {
            const int64_t f = e - nslices;
            const int lane = (int)(f & 63);
            const int64_t r = f >> 6;
            const int js = (int)(r & 1);
            const int64_t t = r >> 1;
            float *o = reinterpret_cast<float *>(B3 + (t * PT + 6 * NDB + 3 * NCB + js) * 256) + lane * 4;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t j = t * 32 + 16 * js + 4 * (lane >> 4) + q;
                o[q] = j < n ? (float)cvec[j] : -__builtin_inff(); // padding: P = 0
            }
        }
    }
}

// The key parts of the F32 median (d > 16, svgd_device.h "F32 pair keys"):
// one thread per (16-row block, 32-k chunk, lane), 8 coordinates split
// into their three bf16 parts (round to nearest: exact, as k_swz_b3).
template <int KP>
__global__ __launch_bounds__(256) void k_swz_keys_b3(const float *__restrict__ xcf, int64_t nblk,
                                                     uint32_t *__restrict__ XK)
{
    constexpr int NDB = KP / 32;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nblk * NDB * 64;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int lane = (int)(e & 63);
        const int64_t r = e >> 6;
        const int db = (int)(r % NDB);
        const int64_t b = r / NDB;
        const float4 *src = reinterpret_cast<const float4 *>(xcf + (16 * b + (lane & 15)) * KP + 32 * db + 8 * (lane >> 4));
        const float4 p = src[0], q = src[1];
        float v[8] = {p.x, p.y, p.z, p.w, q.x, q.y, q.z, q.w};
        uint4 *o = reinterpret_cast<uint4 *>(XK + (b * NDB + db) * 3 * 256) + lane;
#pragma unroll
        for (int part = 0; part < 3; ++part) {
            uint32_t w[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) w[k] = b3_split_pair(v[2 * k], v[2 * k + 1]);
            o[part * 64] = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
}

typedef __bf16 b16x8_t __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f4_t mfma_b3(uint4 a, uint4 b, f4_t c)
{
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b16x8_t, a),
                                                   __builtin_bit_cast(b16x8_t, b), c, 0, 0, 0);
}
// S1V (d = 16 NCB): V holds no column of ones; the row sums sum_j P_ij are
// added on the VALU (padded columns carry c_j = -inf: P = 0).  The part
// products are issued term by term across independent accumulators (the
// Gram chains js x db x rg, the NCB x RG P.V blocks), so no MFMA waits for
// the one before it.  RG row groups of 16 per wave (RG = 2 at large row
// counts, round 6): each tile's column parts, read from LDS once, feed RG
// times the MFMAs -- half the LDS reads and half the barriers per MFMA at
// RG = 2 (2 waves per SIMD at 198 VGPRs instead of 4 at 128).  Measured at
// cfg5 (profiles/r06_b3_rg_il_ab.txt): RG = 2 takes ~15 % more cycles per
// launch but draws less power, so the power-limited chip clocks it ~13 %
// higher -- a wash that moved with the box (step 7.16 vs 7.45 ms on one,
// 7.48 vs 7.14 on another); interleaving the P.V MFMAs with P's VALU
// (sched_group_barrier) recovered ~4 % per clock at RG = 2 and lost 27 % at
// RG = 1.  Default RG = 1; SVGD_PHI_B3_RG=2 selects the other (tests: both
// bit-identical).
template <int KP, int NCB, int NW, bool S1V, int RG = 1>
__global__ __launch_bounds__(64 * NW) void k_phi_b3(
    const uint32_t *__restrict__ B3, const float *__restrict__ crow, const double *__restrict__ a_ptr,
    int64_t row0, int64_t nrows, int64_t ntiles, int d, double inv_n, const double *__restrict__ wv,
    const double *__restrict__ xc, int xc_stride, double *__restrict__ phi, OptArgs opt, int do_opt)
{
    constexpr int NDB = KP / 32, VW = 16 * NCB;
    constexpr int PT = 6 * NDB + 3 * NCB + 2, BUF = PT * 256; // dwords per tile / LDS buffer
    __shared__ __attribute__((aligned(16))) uint32_t sbuf[3 * BUF];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lo = lane & 15, hi = lane >> 4;
    const double a = *a_ptr;
    const float alpha = (float)(2.0 * a * LOG2E);

    const int64_t ibase = row0 + (int64_t)blockIdx.x * (16 * RG * NW) + w * (16 * RG);
    // the Gram's B operand: this wave's RG x 16 rows, from their tiles' XB
    // slices; a row group past the slice (the last block of a rank's rows)
    // loads the slice's first rows instead: valid memory, nothing stored
    uint4 bR[RG][NDB][3];
    float ci[RG];
#pragma unroll
    for (int rg = 0; rg < RG; ++rg) {
        const int64_t ib = ibase + 16 * rg;
        const int64_t ild = ib < row0 + nrows ? ib : row0;
        const int64_t tr = ild / 32;
        const int jsr = (int)((ild / 16) & 1);
#pragma unroll
        for (int db = 0; db < NDB; ++db)
#pragma unroll
            for (int part = 0; part < 3; ++part)
                bR[rg][db][part] = *reinterpret_cast<const uint4 *>(
                    B3 + (tr * PT + (jsr * NDB + db) * 3 + part) * 256 + lane * 4);
        ci[rg] = crow[ild + lo];
    }

    f4_t acc[RG][NCB];
#pragma unroll
    for (int rg = 0; rg < RG; ++rg)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) acc[rg][cb] = f4_t{0.0f, 0.0f, 0.0f, 0.0f};
    float ps[RG]; // S1V: this lane's share of sum_j P_ij, i = lo of each row group
#pragma unroll
    for (int rg = 0; rg < RG; ++rg) ps[rg] = 0.0f;

    auto issue = [&](int64_t t, int b) {
        const char *g = reinterpret_cast<const char *>(B3 + t * BUF);
        char *lb = reinterpret_cast<char *>(sbuf + b * BUF);
        for (int p = w; p < PT; p += NW)
            __builtin_amdgcn_global_load_lds((gbl_void *)(g + p * 1024 + lane * 16), (lds_void *)(lb + p * 1024), 16, 0, 0);
    };
    // part products (A part, B part), smallest first
    constexpr int TA[6] = {1, 0, 2, 0, 1, 0}, TB_[6] = {1, 2, 0, 1, 0, 0};
    // P.V of a tile whose P parts are in aP, its V parts in LDS buffer lv:
    // by V part (l, m, h), each part's terms across the NCB x RG blocks
    uint4 aP[RG][3] = {};
    auto pv_mfma = [&](const uint32_t *lv) {
#pragma unroll
        for (int vp = 2; vp >= 0; --vp) {
            uint4 bV[NCB];
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb)
                bV[cb] = *reinterpret_cast<const uint4 *>(lv + (6 * NDB + 3 * cb + vp) * 256 + lane * 4);
            // P parts paired with V part vp: l -> h; m -> m, h; h -> l, m, h
#pragma unroll
            for (int pp = 2; pp >= 0; --pp) {
                if (pp + vp > 2) continue;
#pragma unroll
                for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
                    for (int rg = 0; rg < RG; ++rg) acc[rg][cb] = mfma_b3(aP[rg][pp], bV[cb], acc[rg][cb]);
            }
        }
    };
    // Software pipeline over three LDS buffers: iteration t issues tile t's
    // Gram MFMAs, then tile t-1's P.V MFMAs (its P parts from the last
    // iteration, its V parts still in buffer (t-1) % 3), and forms tile t's P
    // on the VALU while those are in the matrix pipe.  The DMA of tile t+1
    // goes to buffer (t+1) % 3, whose tile (t-2) every wave finished before
    // this iteration's barrier.  (Round 4 measured a staggered order --
    // waves 4-7 VALU-first -- 6 % slower per clock: profiles/r04_b3_ab.txt.)
    auto gram = [&](const uint32_t *lb, f4_t (&dot)[RG][2][NDB]) {
#pragma unroll
        for (int rg = 0; rg < RG; ++rg)
#pragma unroll
            for (int js = 0; js < 2; ++js)
#pragma unroll
                for (int db = 0; db < NDB; ++db) dot[rg][js][db] = f4_t{0.0f, 0.0f, 0.0f, 0.0f};
        uint4 aX[2][NDB][3];
#pragma unroll
        for (int js = 0; js < 2; ++js)
#pragma unroll
            for (int db = 0; db < NDB; ++db)
#pragma unroll
                for (int part = 0; part < 3; ++part)
                    aX[js][db][part] =
                        *reinterpret_cast<const uint4 *>(lb + ((js * NDB + db) * 3 + part) * 256 + lane * 4);
        // dot[rg][js][db] (4 RG independent chains at KP = 64), term by term
#pragma unroll
        for (int tm = 0; tm < 6; ++tm)
#pragma unroll
            for (int js = 0; js < 2; ++js)
#pragma unroll
                for (int db = 0; db < NDB; ++db)
#pragma unroll
                    for (int rg = 0; rg < RG; ++rg)
                        dot[rg][js][db] = mfma_b3(aX[js][db][TA[tm]], bR[rg][db][TB_[tm]], dot[rg][js][db]);
    };
    // P of a tile from its Gram (its c_j in LDS buffer lb) -> aP, row sums
    auto form_p = [&](const uint32_t *lb, const f4_t (&dot)[RG][2][NDB]) {
        f4_t cj[2];
#pragma unroll
        for (int js = 0; js < 2; ++js)
            cj[js] = *reinterpret_cast<const f4_t *>(lb + (6 * NDB + 3 * NCB + js) * 256 + lane * 4);
#pragma unroll
        for (int rg = 0; rg < RG; ++rg) {
            float pv[8]; // P[i = lo][j = 16js + 4hi + r] at k-slot 4js + r
#pragma unroll
            for (int js = 0; js < 2; ++js) {
                f4_t dd = dot[rg][js][0];
#pragma unroll
                for (int db = 1; db < NDB; ++db) dd += dot[rg][js][db];
#pragma unroll
                for (int r = 0; r < 4; ++r) pv[4 * js + r] = exp2_nonpos(fmaf(alpha, dd[r], ci[rg] + cj[js][r]));
            }
            if (S1V) {
#pragma unroll
                for (int q = 0; q < 8; ++q) ps[rg] += pv[q];
            }
            uint32_t wd[3][4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float x0 = pv[2 * q], x1 = pv[2 * q + 1];
#pragma unroll
                for (int part = 0; part < 3; ++part)
                    wd[part][q] = SVGD_B3_TRUNC ? b3_trunc_pair(x0, x1) : b3_split_pair(x0, x1);
            }
#pragma unroll
            for (int part = 0; part < 3; ++part)
                aP[rg][part] = make_uint4(wd[part][0], wd[part][1], wd[part][2], wd[part][3]);
        }
    };
    auto buf = [&](int64_t t) { return sbuf + (int)(t % 3) * BUF; };
    if (ntiles > 0) issue(0, 0);
    for (int64_t t = 0; t < ntiles; ++t) {
        const int b = (int)(t % 3);
        wait_vmcnt<0>();
        __syncthreads();
        if (t + 1 < ntiles) issue(t + 1, b == 2 ? 0 : b + 1);
        f4_t dot[RG][2][NDB];
        gram(buf(t), dot);
        if (t > 0) pv_mfma(buf(t - 1));
        form_p(buf(t), dot);
    }
    if (ntiles > 0) pv_mfma(buf(ntiles - 1)); // (its buffer is intact: no DMA after it)

    // epilogue (fp64): acc lane map row i = 4 hi + q, column c = lo (+16 cb)
    if (S1V) { // the 4 lane groups' shares of row lo, in a fixed tree
#pragma unroll
        for (int rg = 0; rg < RG; ++rg) {
            ps[rg] += __shfl_xor(ps[rg], 16);
            ps[rg] += __shfl_xor(ps[rg], 32);
        }
    }
    __syncthreads();
    float *sAcc = reinterpret_cast<float *>(sbuf) + w * 16 * RG * (VW + 1);
    static_assert(NW * 16 * RG * (VW + 1) <= 3 * BUF, "epilogue tiles exceed the buffers");
#pragma unroll
    for (int rg = 0; rg < RG; ++rg) {
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
            for (int q = 0; q < 4; ++q) sAcc[(16 * rg + 4 * hi + q) * (VW + 1) + cb * 16 + lo] = acc[rg][cb][q];
        if (S1V && hi == 0) sAcc[(16 * rg + lo) * (VW + 1) + VW] = ps[rg];
    }
    __syncthreads();
    const double two_a = 2.0 * a;
    const int s1c = S1V ? VW : d;
    for (int e = lane; e < 16 * RG * d; e += 64) {
        const int il = e / d, c = e - il * d;
        const int64_t i = ibase + il;
        if (i - row0 < nrows) {
            const double s1 = (double)sAcc[il * (VW + 1) + s1c];
            const double wgt = wv ? wv[i * d + c] : two_a * xc[i * xc_stride + c];
            const double ph = inv_n * ((double)sAcc[il * (VW + 1) + c] + wgt * s1);
            phi[(i - row0) * d + c] = ph;
            if (do_opt) opt_elem(opt, (i - row0) * d + c, ph);
        }
    }
}

// phi_i = (sum_s acc_s + 2a xc_i sum_s acc1_s) / N, partials summed in s order.
// wv (full-matrix scale): 2 M xc_i per particle, in place of 2 a xc_i.
// A block owns phi_red_rows(d) = 256 / (d+1) rows: their (d+1)-element
// partial rows are contiguous in every split s, so each thread sums ONE
// element over the splits (loads issued 8 splits at a time, added in s
// order), the sums go to LDS and phi is written coalesced from LDS.
__host__ __device__ constexpr int phi_red_rows(int d) { return 256 / (d + 1); }
__global__ __launch_bounds__(256) void k_phi_reduce(const double *__restrict__ part,
                                                    const double *__restrict__ rec,
                                                    const double *__restrict__ a_ptr, int64_t row0,
                                                    int64_t nrows, int d, int RS, int S, int64_t ldp,
                                                    double inv_n, const double *__restrict__ wv,
                                                    double *__restrict__ phi, OptArgs opt, int do_opt,
                                                    const int *__restrict__ skip)
{
    if (skip && *skip) return;
    __shared__ double sm[256];
    const int DP = d + 1;
    const int RB = phi_red_rows(d);
    const int64_t rb = (int64_t)blockIdx.x * RB;
    const int rows = (int)min<int64_t>(RB, nrows - rb);
    if (rows <= 0) return;
    // this thread's output element (rows * d < 256: at most one), its
    // weight and optimizer state loaded before the partial sums (one memory
    // round trip fewer)
    const int o = threadIdx.x;
    const bool own = o < rows * d;
    const int r_o = own ? o / d : 0, k_o = own ? o - r_o * d : 0;
    const int64_t li_o = rb + r_o;
    double w_o = 0.0;
    OptIn in_o{0.0, 0.0, 0.0};
    if (own) {
        w_o = wv ? wv[(row0 + li_o) * d + k_o] : 2.0 * (*a_ptr) * rec[(row0 + li_o) * RS + k_o];
        if (do_opt) in_o = opt_load(opt, li_o * d + k_o);
    }
    const int e = threadIdx.x;
    if (e < rows * DP) {
        // 16 splits' loads in flight at once (one memory round trip at S <= 16,
        // the usual case), added in s order
        const double *p = part + rb * DP + e;
        const int64_t st = ldp * DP;
        double acc = 0.0;
        int s = 0;
        for (; s + 16 <= S; s += 16) {
            double v[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = p[(s + q) * st];
#pragma unroll
            for (int q = 0; q < 16; ++q) acc += v[q];
        }
        if (s < S) {
            double v[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = s + q < S ? p[(s + q) * st] : 0.0;
#pragma unroll
            for (int q = 0; q < 16; ++q)
                if (s + q < S) acc += v[q];
        }
        sm[e] = acc;
    }
    __syncthreads();
    if (own) {
        const double ph = inv_n * (sm[r_o * DP + k_o] + w_o * sm[r_o * DP + d]);
        phi[li_o * d + k_o] = ph;
        if (do_opt) opt_apply(opt, li_o * d + k_o, ph, in_o);
    }
}


// Median pair sweep, row-stream form: each wave walks a contiguous run of the
// rank's block tiles (plan.cpp); lane = particle i of the row block, j of the
// column block wave-uniform (scalar loads).  Key = max(|xc_i|^2 + |xc_j|^2 -
// 2 xc_i.xc_j, 0) with the dot as an FMA chain in k order (bit-identical to
// k_sample_keys).  MODE 0 collect, 1 histogram (fallback), 2 debug dump.
constexpr int PR = 4;     // rows per lane of the median sweep
constexpr int CH_MED = 32; // columns per LDS chunk of the median stream

struct TileIt {
    int64_t t, I, J, slot;
    int c;
};

template <int D, int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(D <= 8 ? 4 : 1, 8))) void k_pair_rows(const double *__restrict__ xc, int kp_arg,
                                                  const double *__restrict__ nrm, int64_t n,
                                                  int64_t nb, int64_t t0, int64_t t1,
                                                  SinkCollect sc, SinkHist sh, SinkDebug sd)
{
    // Median records (k_center): [xc (D) | h = -|xc|^2 / 2 | 0..], stride KP.
    // The pair key of rows i, j (every mode, so all passes agree bit for bit):
    //   e_ij = h_j + sum_k xc_ik xc_jk   (fma chain, k ascending)
    //   s_ij = max(fl(-2 h_i - 2 e_ij), 0) = |xc_i - xc_j|^2 up to rounding.
    constexpr int KP = med_rec_stride(D);
    constexpr int CHB = CH_MED * KP * 8; // bytes per column chunk (multiple of 1 KiB)
    constexpr int STG = MODE == 0 ? 256 : 1; // staged keys per wave (MODE 0)
    // per-wave double-buffered column chunks, then (MODE 0) per-wave key
    // staging.  The staging lives inside smem on purpose: a separate
    // __shared__ array makes the compiler drain the in-flight column DMA
    // before every LDS read of the loop.
    __shared__ __attribute__((aligned(16))) char smem[4 * 2 * CHB + (MODE == 0 ? 4 * STG * 8 + NBK * 4 : 0)];
    __shared__ uint32_t sHist[(MODE == 1) ? 2 * RADIX : 1];
    const int tid = threadIdx.x, lane = tid & 63;
    // wave index made provably uniform (wave-uniform tile walk)
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    char *wbuf = smem + w * 2 * CHB;
    (void)kp_arg;
    (void)nrm;

    // MODE 0: each wave appends the keys in [lo, hi) to its own region.  Keys
    // are staged in LDS (asm stores, see lds_store_u64) and flushed right
    // after each column-DMA wait, so the global stores drain during a whole
    // chunk instead of stalling the next vmcnt wait; no LDS atomics.
    uint64_t(*sStage)[STG] = reinterpret_cast<uint64_t(*)[STG]>(smem + 4 * 2 * CHB);
    // (MODE 0) key-range bucket histogram of the staged keys, updated with asm
    // LDS atomics in flush() for the same reason as the staging stores
    uint32_t *sBk = reinterpret_cast<uint32_t *>(smem + 4 * 2 * CHB + (MODE == 0 ? 4 * STG * 8 : 0));
    uint64_t blo = 0;
    double binv = 0.0;
    const int64_t wreg = (int64_t)blockIdx.x * 4 + w;
    int64_t wcnt = 0; // keys written to the region
    int scnt = 0;     // keys staged in sStage[w]
    uint64_t *wregion = MODE == 0 ? sc.region + wreg * sc.cap : nullptr;
    int nsel = 0, shift = 0, hsh = 63;
    uint64_t pfx0 = 0, pfx1 = 0, lo_key = 0, hi_key = 0;
    unsigned long long below = 0; // wave-uniform (scalar) count
    // staged keys: those below lo are counted, those in [lo, hi) appended to
    // the region (and bucketed), the rest dropped; only the occupied 64-key
    // groups are read
    auto flush = [&]() {
        if (scnt == 0) return;
        const int ng = (scnt + 63) >> 6;
        for (int t = 0; t < ng; ++t) {
            const uint64_t key = lds_load_u64_sync(&sStage[w][t * 64 + lane]);
            const bool valid = t * 64 + lane < scnt;
            below += __popcll(__ballot(valid && key < lo_key));
            const bool keep = valid && key >= lo_key && key < hi_key;
            const unsigned long long mk = __ballot(keep);
            if (keep) {
                const int64_t pos = wcnt + __popcll(mk & ((1ull << lane) - 1ull));
                if (pos < sc.cap) wregion[pos] = key;
                if (sc.bpart) lds_add_u32(&sBk[kbucket(key, blo, binv)], 1u);
            }
            wcnt += __popcll(mk);
        }
        scnt = 0;
    };

    double nmax = 0.0;
    if (MODE == 0) {
        lo_key = sc.st->lo_key;
        hi_key = sc.st->hi_key;
        nmax = __longlong_as_double((long long)*sc.nmax_bits);
        blo = lo_key;
        binv = sc.st->binv;
        if (sc.bpart)
            for (int e = tid; e < NBK; e += 256) sBk[e] = 0;
    } else if (MODE == 1) {
        nsel = sh.st->nsel;
        shift = sh.st->shift;
        hsh = shift + sh.st->width;
        pfx0 = sh.st->prefix[0];
        pfx1 = sh.st->prefix[1];
        for (int e = tid; e < 2 * RADIX; e += 256) sHist[e] = 0;
    }
    __syncthreads();

    // keys of non-negative doubles order like the doubles themselves
    const double lo_d = __longlong_as_double((long long)lo_key);
    const double hi_d = hi_key >= 0x7ff0000000000000ull ? __builtin_inf()
                                                        : __longlong_as_double((long long)hi_key);
    // MODE 0 classifies on e directly.  s = fl(n_i - 2e) is monotone in e and
    // within 2^-53 (n_i + 2|e|) <= 2^-51 (n_i + nmax) of n_i - 2e, so with
    // m_i = 2^-48 (n_i + nmax)
    //   e >  TL_i = (n_i - lo + m_i) / 2   =>  s <  lo   (counted)
    //   e <= TH_i = (n_i - hi - m_i) / 2   =>  s >= hi   (ignored)
    // and only the thin band between (the bracket itself) forms s.

    const int64_t W = (int64_t)gridDim.x * 4, gw = (int64_t)blockIdx.x * 4 + w;
    const int64_t T = t1 - t0;
    const int64_t tb = t0 + T * gw / W, te = t0 + T * (gw + 1) / W;
    uint32_t wbelow = 0;          // 32-bit scalar count, flushed per chunk (MODE 0)

    if (tb < te) {
        const int64_t H = (nb - 1) / 2;
        // flat stream of (tile, 32-column chunk) items; the DMA of item q+1
        // into this wave's other LDS buffer overlaps the compute of item q
        TileIt it;
        tile_coords(nb, tb, &it.I, &it.J);
        it.t = tb;
        it.slot = (it.J - it.I + nb) % nb;
        it.c = 0;
        auto advance = [&](TileIt &x) {
            const int64_t jb = x.J * PBLK, je = min(jb + PBLK, n);
            if (++x.c * CH_MED < je - jb) return;
            x.c = 0;
            ++x.t;
            ++x.slot;
            const int64_t cntI = ((nb & 1) == 0 && x.I < nb / 2) ? H + 2 : H + 1;
            if (x.slot == cntI) {
                ++x.I;
                x.slot = 0;
            }
            x.J = x.slot == 0 ? x.I : (x.I + x.slot) % nb;
        };
        auto src = [&](const TileIt &x) {
            return reinterpret_cast<const char *>(xc + (x.J * PBLK + x.c * CH_MED) * KP);
        };
        dma_to_lds<CHB>(src(it), wbuf, lane);
        int64_t curI = -1;
        double xi[PR][D], ni[PR], TL[PR], TH[PR];
        // row index / validity recomputed where needed (the diagonal tiles and
        // the rare key path) instead of held in 12 VGPRs across the loop
        auto irow = [&](int r) -> int64_t { return curI * PBLK + 64 * r + lane; };
        auto ivalid = [&](int r) -> bool { return irow(r) < n; };
        for (int q = 0; it.t < te; ++q) {
            TileIt nx = it;
            advance(nx);
            if (nx.t < te) {
                dma_to_lds<CHB>(src(nx), wbuf + ((q + 1) & 1) * CHB, lane);
                wait_vmcnt<CHB / 1024>();
            } else {
                wait_vmcnt<0>();
            }
            if constexpr (MODE == 0) {
                flush();
                below += wbelow; // a chunk adds < 2^14 to the 32-bit count
                wbelow = 0;
            }
            const int64_t I = it.I, J = it.J;
            if (I != curI) {
#pragma unroll
                for (int r = 0; r < PR; ++r) {
                    const int64_t ir = I * PBLK + 64 * r + lane;
                    const bool iv = ir < n;
                    const int64_t ic = iv ? ir : n - 1;
#pragma unroll
                    for (int k = 0; k < D; ++k) xi[r][k] = xc[ic * KP + k];
                    ni[r] = -2.0 * xc[ic * KP + D];
                    if constexpr (MODE == 0) {
                        const double m = 0x1p-48 * (ni[r] + nmax);
                        TL[r] = lo_key == 0 ? __builtin_inf() : 0.5 * (ni[r] - lo_d + m);
                        TH[r] = 0.5 * (ni[r] - hi_d - m); // -inf when hi is +inf
                        if (!iv) TL[r] = TH[r] = __builtin_inf(); // never counted
                    }
                }
                // row registers complete here (rare: once per row block), not
                // at their first use inside the column loop
                wait_vmcnt<0>();
                curI = I;
            }
            const bool diag = I == J;
            const int64_t jb = J * PBLK + it.c * CH_MED;
            const int cnt = (int)min<int64_t>(CH_MED, n - jb);
            const double *cb = reinterpret_cast<const double *>(wbuf + (q & 1) * CHB);
            // off-diagonal tiles (all but 1 in H+1): every valid row counts
            // the bracket band of one column: form the keys of the rows in mcs
            auto band = [&](const double(&ev)[PR], const unsigned long long(&mcs)[PR]) {
#pragma unroll
                for (int r = 0; r < PR; ++r) {
                    // every key of the threshold band is staged as is; flush()
                    // classifies it exactly (below lo / in [lo, hi) / above)
                    // once per 64 staged keys instead of once per band row
                    const unsigned long long mc = mcs[r];
                    if (!mc) continue;
                    if (scnt + 64 > STG) flush(); // rare: > STG-64 keys in a chunk
                    if ((mc >> lane) & 1ull)
                        lds_store_u64(&sStage[w][scnt + __popcll(mc & ((1ull << lane) - 1ull))],
                                      key_of(fmax(fma(-2.0, ev[r], ni[r]), 0.0)));
                    scnt += __popcll(mc);
                }
            };
            auto columns = [&](auto diag_tag) {
                constexpr bool DIAG = decltype(diag_tag)::value;
                // MODE 0 off-diagonal tiles (the bulk): the column record of jj+1
                // is read from LDS while column jj is classified (the read past
                // the chunk's last column stays inside smem and is discarded)
                constexpr bool PIPE = false; // (MODE == 0 && !DIAG: measured no faster)
                auto column = [&](const double(&cr)[D + 1], const int64_t j) {
                    const double *xj = cr;
                    const double hj = cr[D];
                    // all rows' chains first (independent, interleaved), then
                    // the classification: no branch between the FMA chains
                    double ev[PR];
#pragma unroll
                    for (int r = 0; r < PR; ++r) {
                        ev[r] = hj;
#pragma unroll
                        for (int k = 0; k < D; ++k) ev[r] = fma(xi[r][k], xj[k], ev[r]);
                    }
                    if constexpr (MODE == 0) {
                        // two f64 compares per pair.  Off-diagonal tiles count
                        // per lane (invalid rows have TL = TH = +inf) and take
                        // one wave-uniform branch per column; diagonal tiles
                        // (1 in H+1) use SGPR masks for the i < j condition.
                        unsigned long long mcs[PR];
#pragma unroll
                        for (int r = 0; r < PR; ++r) {
                            const unsigned long long ml = __ballot(ev[r] > TL[r]);
                            const unsigned long long mh = __ballot(ev[r] > TH[r]);
                            if constexpr (DIAG) {
                                const unsigned long long vm = __ballot(ivalid(r) && irow(r) < j);
                                below += __popcll(ml & vm);
                                mcs[r] = mh & ~ml & vm;
                            } else {
                                // invalid rows: TL = TH = +inf, so no mask
                                wbelow += (uint32_t)__popcll(ml);
                                mcs[r] = mh & ~ml;
                            }
                        }
                        unsigned long long anyc = 0;
#pragma unroll
                        for (int r = 0; r < PR; ++r) anyc |= mcs[r];
                        if (anyc) band(ev, mcs);
                    }
#pragma unroll
                    for (int r = 0; r < PR; ++r) {
                        const double e = ev[r];
                        const bool valid = ivalid(r) && (!DIAG || irow(r) < j);
                        if constexpr (MODE == 0) {
                            (void)e;
                            (void)valid;
                        } else {
                            const double sk = fmax(fma(-2.0, e, ni[r]), 0.0);
                            if (MODE == 1) {
                                if (valid) {
                                    const uint64_t key = key_of(sk);
                                    const uint32_t dg = (uint32_t)((key >> shift) & (RADIX - 1));
                                    if (hsh >= 64 || (key >> hsh) == (pfx0 >> hsh))
                                        atomicAdd(&sHist[dg], 1u);
                                    if (nsel > 1 && (hsh >= 64 || (key >> hsh) == (pfx1 >> hsh)))
                                        atomicAdd(&sHist[RADIX + dg], 1u);
                                }
                            } else {
                                if (valid) {
                                    const int64_t i = irow(r);
                                    const int64_t a = i < j ? i : j, b = i < j ? j : i;
                                    sd.out[a * (2 * sd.n - a - 1) / 2 + (b - a - 1)] = sk;
                                }
                            }
                        }
                    }
                };
                auto load = [&](double(&cr)[D + 1], int jj) {
#pragma unroll
                    for (int k = 0; k <= D; ++k) cr[k] = cb[jj * KP + k]; // LDS broadcast
                };
                if constexpr (PIPE) {
                    double qa[D + 1], qb[D + 1];
                    load(qa, 0);
                    __builtin_amdgcn_s_waitcnt(0xC07F); // lgkmcnt(0) before the loop head
                    for (int jj = 0; jj < cnt; jj += 2) {
                        load(qb, jj + 1);
                        __builtin_amdgcn_sched_barrier(0);
                        column(qa, jb + jj);
                        __builtin_amdgcn_sched_barrier(0);
                        if (jj + 1 >= cnt) break;
                        load(qa, jj + 2);
                        __builtin_amdgcn_sched_barrier(0);
                        column(qb, jb + jj + 1);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                } else {
                    // 2 columns per iteration (one loop test per two), then the rest
                    int jj = 0;
                    for (; jj + 2 <= cnt; jj += 2) {
                        double cr[D + 1];
                        load(cr, jj);
                        column(cr, jb + jj);
                        load(cr, jj + 1);
                        column(cr, jb + jj + 1);
                    }
                    if (jj < cnt) {
                        double cr[D + 1];
                        load(cr, jj);
                        column(cr, jb + jj);
                    }
                }
            };
            if (diag)
                columns(std::true_type{});
            else
                columns(std::false_type{});
            it = nx;
        }
    }

    if constexpr (MODE == 0) {
        flush();
        below += wbelow;
        if (lane == 0) {
            sc.below_out[wreg] = below;
            sc.count_out[wreg] = (uint32_t)min<int64_t>(wcnt, 0xffffffffll);
        }
        if (sc.bpart) {
            lgkm_wait(); // this wave's asm bucket atomics
            __syncthreads();
            for (int e = tid; e < NBK; e += 256) sc.bpart[(int64_t)blockIdx.x * NBK + e] = sBk[e];
        }
    } else if (MODE == 1) {
        __syncthreads();
        for (int e = tid; e < 2 * RADIX; e += 256)
            if (sHist[e]) atomicAdd(&sh.ghist[e], (unsigned long long)sHist[e]);
    }
}

// =========================================== full-matrix kernel scale ==
// k(x, x') = exp(-(x-x')^T M (x-x')) with M = L L^T (GaussianRBFKernel.hpp:
// 75-81; M from the Hessian heuristic :189-210 or a user constant).  The phi
// kernels run unchanged on z = L^T xc with a = 1 (|z_i - z_j|^2 is the
// M-distance); V_j = G_j - 2 M xc_j and the reduce adds 2 M xc_i sum_j K_ij.
//
// One thread: M = factor * src (symmetrised) and a factor M = L S L^T with
// S = diag(sgn): the Cholesky factor (sgn = +1) when M is positive definite,
// else (d <= ROWS_MAX_D) L = Q |Lambda|^(1/2), sgn = sign(Lambda) from a cyclic
// Jacobi eigendecomposition -- the reference evaluates (x-x')^T M (x-x')
// for any symmetric M (GaussianRBFKernel.hpp:75-81, 189-210), and the
// sum of -Hessians of a Gaussian mixture can be indefinite between modes.
// err = 0 (positive definite), 2 (indefinite: factored for d <= 16, else not),
// 1 (non-finite M or no convergence).  a_eff = 1 for the phi kernels.
// work: 2 d^2 doubles (Jacobi A and V).
__global__ void k_scale_factor(const double *__restrict__ src, double factor, int d,
                               double *__restrict__ M, double *__restrict__ L,
                               double *__restrict__ sgn, double *__restrict__ work,
                               double *__restrict__ scal, int *__restrict__ err)
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    scal[0] = 1.0;
    scal[1] = __builtin_nan("");
    double nrm = 0.0;
    for (int r = 0; r < d; ++r)
        for (int c = 0; c < d; ++c) {
            const double m = factor * 0.5 * (src[r * d + c] + src[c * d + r]);
            M[r * d + c] = m;
            nrm += m * m;
        }
    if (!(nrm < __builtin_inf())) {
        *err = 1;
        return;
    }
    bool pd = true;
    for (int j = 0; j < d && pd; ++j) {
        double s = M[j * d + j];
        for (int k = 0; k < j; ++k) s -= L[j * d + k] * L[j * d + k];
        if (!(s > 0.0)) {
            pd = false;
            break;
        }
        const double ljj = sqrt(s);
        L[j * d + j] = ljj;
        for (int i = j + 1; i < d; ++i) {
            double t = M[i * d + j];
            for (int k = 0; k < j; ++k) t -= L[i * d + k] * L[j * d + k];
            L[i * d + j] = t / ljj;
        }
        for (int c = j + 1; c < d; ++c) L[j * d + c] = 0.0;
        sgn[j] = 1.0;
    }
    if (pd) {
        *err = 0;
        return;
    }
    if (d > ROWS_MAX_D) { // the MFMA tile kernels take positive definite M only
        *err = 2;
        return;
    }
    double *A = work, *V = work + d * d;
    for (int r = 0; r < d; ++r)
        for (int c = 0; c < d; ++c) {
            A[r * d + c] = M[r * d + c];
            V[r * d + c] = r == c ? 1.0 : 0.0;
        }
    bool conv = false;
    for (int sweep = 0; sweep < 60 && !conv; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < d; ++p)
            for (int q = p + 1; q < d; ++q) off += A[p * d + q] * A[p * d + q];
        if (off <= 1e-34 * nrm) {
            conv = true;
            break;
        }
        for (int p = 0; p < d; ++p)
            for (int q = p + 1; q < d; ++q) {
                const double apq = A[p * d + q];
                if (apq == 0.0) continue;
                const double theta = (A[q * d + q] - A[p * d + p]) / (2.0 * apq);
                const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), sn = t * c;
                for (int k = 0; k < d; ++k) { // A <- A J (columns p, q)
                    const double akp = A[k * d + p], akq = A[k * d + q];
                    A[k * d + p] = c * akp - sn * akq;
                    A[k * d + q] = sn * akp + c * akq;
                }
                for (int k = 0; k < d; ++k) { // A <- J^T A (rows p, q)
                    const double apk = A[p * d + k], aqk = A[q * d + k];
                    A[p * d + k] = c * apk - sn * aqk;
                    A[q * d + k] = sn * apk + c * aqk;
                }
                for (int k = 0; k < d; ++k) { // V <- V J
                    const double vkp = V[k * d + p], vkq = V[k * d + q];
                    V[k * d + p] = c * vkp - sn * vkq;
                    V[k * d + q] = sn * vkp + c * vkq;
                }
            }
    }
    if (!conv) {
        *err = 1;
        return;
    }
    for (int k = 0; k < d; ++k) {
        const double lam = A[k * d + k];
        const double sq = sqrt(fabs(lam));
        sgn[k] = lam > 0.0 ? 1.0 : (lam < 0.0 ? -1.0 : 0.0);
        for (int l = 0; l < d; ++l) L[l * d + k] = V[l * d + k] * sq; // z_k = sum_l L[l][k] x_l
    }
    *err = 2;
}

// Row-stream records for the matrix scale: rec_j = [z_j | G_j - 2 M xc_j |
// -4096 log2e z_j^T S z_j | 0..], wv_j = 2 M xc_j (z = L^T xc, M = L S L^T).
__global__ void k_prep_rec_mat(const double *__restrict__ xc, const double *__restrict__ G,
                               const double *__restrict__ M, const double *__restrict__ L,
                               const double *__restrict__ sgn, int64_t n, int64_t np, int d, int KP,
                               int RS, double *__restrict__ rec, double *__restrict__ wv)
{
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < np;
         j += (int64_t)gridDim.x * blockDim.x) {
        const bool live = j < n;
        double *r = rec + j * RS;
        double zz = 0.0;
        for (int k = 0; k < d; ++k) {
            double z = 0.0, mx = 0.0;
            if (live)
                for (int l = 0; l < d; ++l) {
                    const double x = xc[j * KP + l];
                    z = fma(L[l * d + k], x, z);
                    mx = fma(M[k * d + l], x, mx);
                }
            r[k] = z;
            r[d + k] = live ? G[j * d + k] - 2.0 * mx : 0.0;
            wv[j * d + k] = 2.0 * mx;
            zz = fma(sgn[k] * z, z, zz);
        }
        r[2 * d] = live ? -4096.0 * LOG2E * zz : 0.0;
        for (int k = 2 * d + 1; k < RS; ++k) r[k] = 0.0;
    }
}

// MFMA path (d > 16): zc = [z | 0..] (stride KP), V = [G - 2 M xc, 1, 0..],
// cvec = -log2e |z|^2, wv = 2 M xc.
__global__ void k_prep_v_mat(const double *__restrict__ xc, const double *__restrict__ G,
                             const double *__restrict__ M, const double *__restrict__ L,
                             int64_t n, int64_t np, int d, int KP, int VW,
                             double *__restrict__ zc, double *__restrict__ V,
                             double *__restrict__ cvec, double *__restrict__ wv)
{
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < np;
         j += (int64_t)gridDim.x * blockDim.x) {
        const bool live = j < n;
        double zz = 0.0;
        for (int k = 0; k < KP; ++k) {
            double z = 0.0, mx = 0.0;
            if (live && k < d)
                for (int l = 0; l < d; ++l) {
                    const double x = xc[j * KP + l];
                    z = fma(L[l * d + k], x, z);
                    mx = fma(M[k * d + l], x, mx);
                }
            zc[j * KP + k] = z;
            zz = fma(z, z, zz);
            if (k < d) wv[j * d + k] = 2.0 * mx;
            if (k < VW) V[j * VW + k] = live && k < d ? G[j * d + k] - 2.0 * mx : 0.0;
        }
        for (int k = KP; k < VW; ++k) V[j * VW + k] = 0.0;
        if (d < VW) V[j * VW + d] = live ? 1.0 : 0.0;
        cvec[j] = live ? -LOG2E * zz : 0.0;
    }
}

// ================================================ device log-gradient ==
// grad log p for the built-in Gaussian-sum model (MultivariateNormal.hpp:56-61,
// Model::operator+ Model.hpp:55-92): p = sum_c exp(-q_c / 2), q_c = (x-mu_c)^T
// P_c (x-mu_c); grad = sum_c w_c (-P_c (x - mu_c)) / sum_c w_c with
// w_c = exp(-(q_c - q_min) / 2).  Same operation order as host_models.cpp.
// One thread per particle row; mu and P are read through the cache.
template <int D>
__global__ __launch_bounds__(256) void k_gauss_grad(const double *__restrict__ X, int64_t rows,
                                                    int d_rt, int k, const double *__restrict__ mu,
                                                    const double *__restrict__ prec,
                                                    double *__restrict__ G)
{
    constexpr int DM = D > 0 ? D : 64;
    const int d = D > 0 ? D : d_rt;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows) return;
    double x[DM], acc[DM], diff[DM];
    for (int r = 0; r < d; ++r) {
        x[r] = X[i * d + r];
        acc[r] = 0.0;
    }
    // pass 1: q_c and q_min (the host keeps every g_c; here g_c is recomputed
    // in pass 2 to keep registers bounded -- identical arithmetic)
    double qmin = __builtin_inf();
    for (int c = 0; c < k; ++c) {
        const double *P = prec + (size_t)c * d * d, *m = mu + (size_t)c * d;
        for (int r = 0; r < d; ++r) diff[r] = x[r] - m[r];
        double qq = 0.0;
        for (int r = 0; r < d; ++r) {
            double s = 0.0;
            for (int l = 0; l < d; ++l) s += P[r * d + l] * diff[l];
            qq += diff[r] * s;
        }
        qmin = fmin(qmin, 0.5 * qq);
    }
    double wsum = 0.0;
    for (int c = 0; c < k; ++c) {
        const double *P = prec + (size_t)c * d * d, *m = mu + (size_t)c * d;
        for (int r = 0; r < d; ++r) diff[r] = x[r] - m[r];
        double qq = 0.0;
        double g[DM];
        for (int r = 0; r < d; ++r) {
            double s = 0.0;
            for (int l = 0; l < d; ++l) s += P[r * d + l] * diff[l];
            g[r] = -s;
            qq += diff[r] * s;
        }
        const double w = exp(-(0.5 * qq - qmin));
        wsum += w;
        for (int r = 0; r < d; ++r) acc[r] += w * g[r];
    }
    for (int r = 0; r < d; ++r) G[i * d + r] = acc[r] / wsum;
}

// ============================================================ launchers ==

#define SVGD_ROWS_CASE(Dv)                                                                   \
    case Dv:                                                                                 \
        if (kind == 0 && R == 1)                                                             \
            hipLaunchKernelGGL((k_phi_rows<Dv, 1>), dim3(grid), dim3(256), 0, stream,   \
                               rec, a_ptr, row0, nrows, n, S, part, ldp, sgn, nmax);               \
        else if (kind == 0 && R == 2)                                                        \
            hipLaunchKernelGGL((k_phi_rows<Dv, 2>), dim3(grid), dim3(256), 0, stream,   \
                               rec, a_ptr, row0, nrows, n, S, part, ldp, sgn, nmax);               \
        else if (kind == 0)                                                                  \
            hipLaunchKernelGGL((k_phi_rows<Dv, 4>), dim3(grid), dim3(256), 0, stream,   \
                               rec, a_ptr, row0, nrows, n, S, part, ldp, sgn, nmax);               \
        else if (kind == 10)                                                                 \
            hipLaunchKernelGGL((k_pair_rows<Dv, 0>), dim3(grid), dim3(256), 0, stream, xc, KP, \
                               nrm, n, nb, t0, t1, sc, sh, sd);                              \
        else if (kind == 11)                                                                 \
            hipLaunchKernelGGL((k_pair_rows<Dv, 1>), dim3(grid), dim3(256), 0, stream, xc, KP, \
                               nrm, n, nb, t0, t1, sc, sh, sd);                              \
        else                                                                                 \
            hipLaunchKernelGGL((k_pair_rows<Dv, 2>), dim3(grid), dim3(256), 0, stream, xc, KP, \
                               nrm, n, nb, t0, t1, sc, sh, sd);                              \
        break;

static hipError_t launch_rows_kernel(int kind, int D, int R, int grid, const double *rec,
                                     const double *a_ptr, int64_t row0, int64_t nrows, int64_t n,
                                     int S, double *part, int64_t ldp, const double *sgn,
                                     const unsigned long long *nmax, const double *xc, int KP,
                                     const double *nrm, int64_t nb, int64_t t0, int64_t t1,
                                     SinkCollect sc, SinkHist sh, SinkDebug sd, hipStream_t stream)
{
    switch (D) {
        SVGD_ROWS_CASE(1)
        SVGD_ROWS_CASE(2)
        SVGD_ROWS_CASE(3)
        SVGD_ROWS_CASE(4)
        SVGD_ROWS_CASE(5)
        SVGD_ROWS_CASE(6)
        SVGD_ROWS_CASE(7)
        SVGD_ROWS_CASE(8)
        SVGD_ROWS_CASE(9)
        SVGD_ROWS_CASE(10)
        SVGD_ROWS_CASE(11)
        SVGD_ROWS_CASE(12)
        SVGD_ROWS_CASE(13)
        SVGD_ROWS_CASE(14)
        SVGD_ROWS_CASE(15)
        SVGD_ROWS_CASE(16)
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_prep_rec(const double *xc, const double *G, const double *nrm,
                           const double *a_ptr, int64_t n, int64_t np, int d, int KP, int RS,
                           double *rec, hipStream_t stream)
{
    int64_t g = (np * RS + 255) / 256;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_prep_rec, dim3(g), dim3(256), 0, stream, xc, G, nrm, a_ptr, n, np, d, KP,
                       RS, rec);
    return hipGetLastError();
}

// kind 2: k_phi_rows with 8 waves, the 8192-entry table and the columns split
// over the 8 waves (WC = 8: one 64 R-row group per work-group); R = 4 for
// d <= 8, 2 above (the register budget)
bool phi_rows_t8k_supported(int d, int R) { return d >= 1 && d <= 16 && R == (d <= 8 ? 4 : 2); }
int phi_rows_t8k_rows(int R) { return (T8K_NW / T8K_WC) * 64 * R; }
#define SVGD_T8K_KERNEL(Dv) k_phi_rows<Dv, ((Dv) <= 8 ? 4 : 2), T8K_NW, 8192, T8K_WC>
#define SVGD_T8K_CASE(Dv)                                                                       \
    case Dv:                                                                                    \
        hipLaunchKernelGGL((SVGD_T8K_KERNEL(Dv)), dim3(grid), dim3(T8K_NW * 64), 0, stream, rec, \
                           a_ptr, row0, nrows, n, S, part, ldp, sgn, nmax);                     \
        break;
static hipError_t launch_rows_t8k(int d, int grid, const double *rec, const double *a_ptr,
                                  int64_t row0, int64_t nrows, int64_t n, int S, double *part,
                                  int64_t ldp, const double *sgn, const unsigned long long *nmax,
                                  hipStream_t stream)
{
    switch (d) {
        SVGD_T8K_CASE(1) SVGD_T8K_CASE(2) SVGD_T8K_CASE(3) SVGD_T8K_CASE(4)
        SVGD_T8K_CASE(5) SVGD_T8K_CASE(6) SVGD_T8K_CASE(7) SVGD_T8K_CASE(8)
        SVGD_T8K_CASE(9) SVGD_T8K_CASE(10) SVGD_T8K_CASE(11) SVGD_T8K_CASE(12)
        SVGD_T8K_CASE(13) SVGD_T8K_CASE(14) SVGD_T8K_CASE(15) SVGD_T8K_CASE(16)
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_phi_rows(int d, int R, const double *rec, const double *a_ptr,
                           int64_t row0, int64_t nrows, int64_t n, int S, double *part,
                           int64_t ldp, double inv_n, const double *wv, const double *sgn,
                           const unsigned long long *nmax_bits, double *phi, const OptArgs *opt,
                           hipStream_t stream, hipEvent_t ev_mid, int kind, const int *skip, bool reduce)
{
    if (nrows <= 0) {
        if (ev_mid) return hipEventRecord(ev_mid, stream);
        return hipSuccess;
    }
    const int rows_wg = kind == 2 ? phi_rows_t8k_rows(R) : 256 * R;
    const int grid = (int)(((nrows + rows_wg - 1) / rows_wg) * S);
    hipError_t e = kind == 2 ? launch_rows_t8k(d, grid, rec, a_ptr, row0, nrows, n, S, part, ldp, sgn,
                                               nmax_bits, stream)
                             : launch_rows_kernel(0, d, R, grid, rec, a_ptr, row0, nrows, n, S, part, ldp, sgn,
                                      nmax_bits, nullptr, 0, nullptr, 0, 0, 0, SinkCollect{}, SinkHist{},
                                      SinkDebug{}, stream);
    if (e != hipSuccess) return e;
    if (ev_mid && (e = hipEventRecord(ev_mid, stream)) != hipSuccess) return e;
    if (!reduce) return hipSuccess;
    if (d > 16) return hipErrorInvalidValue; // k_phi_reduce's LDS holds d + 1 <= 17
    const int64_t g = (nrows + phi_red_rows(d) - 1) / phi_red_rows(d);
    hipLaunchKernelGGL(k_phi_reduce, dim3(g), dim3(256), 0, stream, part, rec, a_ptr, row0, nrows,
                       d, phi_rec_stride(d), S, ldp, inv_n, wv, phi, opt ? *opt : OptArgs{},
                       opt ? 1 : 0, skip);
    return hipGetLastError();
}

hipError_t launch_pair_rows(int d, int KP, int mode, int grid, const double *xc, const double *nrm,
                            const float *xf, const unsigned long long *nmax_bits,
                            int64_t n, int64_t nb, int64_t t0, int64_t t1, uint64_t *regions,
                            int64_t cap, uint32_t *counts, unsigned long long *below,
                            const SelState *st, unsigned long long *ghist, uint32_t *bpart,
                            double *dbg_out, hipStream_t stream)
{
    if (grid <= 0 || t1 <= t0) return hipSuccess;
    if (mode == 0 && !nmax_bits) return hipErrorInvalidValue;
    SinkCollect sc{st, regions, cap, counts, below, xf, nmax_bits, mode == 0 ? bpart : nullptr};
    SinkHist sh{st, ghist};
    SinkDebug sd{dbg_out, n};
    return launch_rows_kernel(10 + mode, d, 1, grid, nullptr, nullptr, 0, 0, n, 1, nullptr, 0, nullptr, nullptr, xc,
                              KP, nrm, nb, t0, t1, sc, sh, sd, stream);
}

// fp64: 8-wave blocks, 2 per CU (76 KB LDS at d = 64), column tile prefetched
// into registers; fp32 (small-N fallback of SVGD_F32): 4 waves, synchronous
// staging.  SVGD_PHI_NW / _PRE / _WPE override at build time for measurements.
#ifndef SVGD_PHI_NW
#define SVGD_PHI_NW 8
#endif
#ifndef SVGD_PHI_PRE
#define SVGD_PHI_PRE 1
#endif
template <class T> struct PhiCfg {
    static constexpr int NW = 4;
    static constexpr bool PRE = false;
};
template <> struct PhiCfg<double> {
    static constexpr int NW = SVGD_PHI_NW;
    static constexpr bool PRE = SVGD_PHI_PRE;
};

template <class T, int KPv, int NCBv, bool S1V>
static hipError_t launch_phi_tile(const T *xg, const T *cvec, const T *V, const double *a_ptr,
                                  int64_t row0, int64_t nrows, int64_t ntiles_j, int64_t n, int d,
                                  double inv_n, const double *wv, const double *xc, double *phi,
                                  hipStream_t stream)
{
    constexpr int NW = PhiCfg<T>::NW;
    const int64_t grid = (nrows + 16 * NW - 1) / (16 * NW);
    hipLaunchKernelGGL((k_phi<T, KPv, NCBv, NW, PhiCfg<T>::PRE, S1V>), dim3(grid), dim3(64 * NW), 0,
                       stream, xg, cvec, V, a_ptr, row0, nrows, ntiles_j, n, d, inv_n, wv, xc, phi);
    return hipGetLastError();
}
#define SVGD_PHI_CASE(KPv, NCBv)                                                             \
    if (KP == KPv && NCB == NCBv)                                                            \
        return launch_phi_tile<T, KPv, NCBv, false>(xg, cvec, V, a_ptr, row0, nrows, ntiles_j, \
                                                    n, d, inv_n, wv, xc, phi, stream);
#define SVGD_PHI_CASE_S1V(KPv, NCBv)                                                         \
    if (KP == KPv && NCB == NCBv && d == 16 * NCBv)                                          \
        return launch_phi_tile<T, KPv, NCBv, true>(xg, cvec, V, a_ptr, row0, nrows, ntiles_j,  \
                                                   n, d, inv_n, wv, xc, phi, stream);

// S1V tiles (d = 16 NCB > 16: fp64, and F32 under the bf16 matrix-core phi)
bool phi_tile_s1v(int d) { return d > 16 && d <= 64 && d % 16 == 0; }
void phi_tile_cfg(bool f64, int *nw, int *pre)
{
    *nw = f64 ? PhiCfg<double>::NW : PhiCfg<float>::NW;
    *pre = f64 ? PhiCfg<double>::PRE : PhiCfg<float>::PRE;
}

template <class T>
static hipError_t launch_phi_t(int KP, int NCB, const T *xg, const T *cvec, const T *V,
                               const double *a_ptr, int64_t row0, int64_t nrows, int64_t ntiles_j,
                               int64_t n, int d, double inv_n, const double *wv, const double *xc,
                               double *phi, hipStream_t stream)
{
    if (nrows <= 0) return hipSuccess;
    SVGD_PHI_CASE_S1V(32, 2)
    SVGD_PHI_CASE_S1V(64, 3)
    SVGD_PHI_CASE_S1V(64, 4)
    SVGD_PHI_CASE(4, 1)
    SVGD_PHI_CASE(8, 1)
    SVGD_PHI_CASE(12, 1)
    SVGD_PHI_CASE(16, 1)
    SVGD_PHI_CASE(16, 2)
    SVGD_PHI_CASE(32, 2)
    SVGD_PHI_CASE(32, 3)
    SVGD_PHI_CASE(64, 4)
    SVGD_PHI_CASE(64, 5)
    return hipErrorInvalidValue;
}
#undef SVGD_PHI_CASE
#undef SVGD_PHI_CASE_S1V

hipError_t launch_phi(int KP, int NCB, const double *xc, const double *cvec, const double *V,
                      const double *a_ptr, int64_t row0, int64_t nrows, int64_t ntiles_j, int64_t n,
                      int d, double inv_n, const double *wv, double *phi, hipStream_t stream)
{
    return launch_phi_t<double>(KP, NCB, xc, cvec, V, a_ptr, row0, nrows, ntiles_j, n, d, inv_n,
                                wv, xc, phi, stream);
}

hipError_t launch_phi_f32(int KP, int NCB, const float *xg, const float *cvec, const float *V,
                          const double *a_ptr, int64_t row0, int64_t nrows, int64_t ntiles_j,
                          int64_t n, int d, double inv_n, const double *wv, const double *xc,
                          double *phi, hipStream_t stream)
{
    return launch_phi_t<float>(KP, NCB, xg, cvec, V, a_ptr, row0, nrows, ntiles_j, n, d, inv_n, wv,
                               xc, phi, stream);
}

#define SVGD_TILE_CASE(KPv)                                                                  \
    if (KP == KPv) {                                                                         \
        if (mode == 0)                                                                       \
            hipLaunchKernelGGL((k_pair_tiles<T, KPv, 0>), dim3(grid), dim3(256), 0, stream,  \
                               xc, nrm, n, nb, t0, t1, sc, sh, sd, xk);                          \
        else if (mode == 1)                                                                  \
            hipLaunchKernelGGL((k_pair_tiles<T, KPv, 1>), dim3(grid), dim3(256), 0, stream,  \
                               xc, nrm, n, nb, t0, t1, sc, sh, sd, xk);                          \
        else if (mode == 2)                                                                  \
            hipLaunchKernelGGL((k_pair_tiles<T, KPv, 2>), dim3(grid), dim3(256), 0, stream,  \
                               xc, nrm, n, nb, t0, t1, sc, sh, sd, xk);                          \
        else                                                                                 \
            hipLaunchKernelGGL((k_pair_tiles<T, KPv, 3>), dim3(grid), dim3(256), 0, stream,  \
                               xc, nrm, n, nb, t0, t1, sc, sh, sd, xk);                          \
        return hipGetLastError();                                                            \
    }

template <class T>
static hipError_t launch_pair_tiles_t(int KP, int mode, int grid, const T *xc, const T *nrm,
                                      int64_t n, int64_t nb, int64_t t0, int64_t t1,
                                      uint64_t *regions, int64_t cap, uint32_t *counts,
                                      unsigned long long *below, const SelState *st,
                                      unsigned long long *ghist, uint32_t *bpart, double *dbg_out,
                                      hipStream_t stream, uint64_t *sample_out = nullptr,
                                      const uint32_t *xk = nullptr)
{
    if (grid <= 0 || t1 <= t0) return hipSuccess;
    // F32 keys at KP 32 / 64 are the bf16 part-product keys: their parts are required
    if (sizeof(T) == 4 && kb3_keys(KP) && !xk) return hipErrorInvalidValue;
    SinkCollect sc{st, regions, cap, counts, below, nullptr, nullptr, mode == 0 ? bpart : nullptr};
    SinkHist sh{st, ghist};
    SinkDebug sd{dbg_out, n, sample_out};
    SVGD_TILE_CASE(4)
    SVGD_TILE_CASE(8)
    SVGD_TILE_CASE(12)
    SVGD_TILE_CASE(16)
    SVGD_TILE_CASE(32)
    SVGD_TILE_CASE(64)
    return hipErrorInvalidValue;
}
#undef SVGD_TILE_CASE

hipError_t launch_pair_tiles(int KP, int mode, int grid, const double *xc, const double *nrm,
                             int64_t n, int64_t nb, int64_t t0, int64_t t1, uint64_t *regions,
                             int64_t cap, uint32_t *counts, unsigned long long *below,
                             const SelState *st, unsigned long long *ghist, uint32_t *bpart,
                             double *dbg_out, hipStream_t stream)
{
    return launch_pair_tiles_t<double>(KP, mode, grid, xc, nrm, n, nb, t0, t1, regions, cap,
                                       counts, below, st, ghist, bpart, dbg_out, stream);
}

hipError_t launch_pair_tiles_f32(int KP, int mode, int grid, const float *xc, const float *nrm,
                                 int64_t n, int64_t nb, int64_t t0, int64_t t1, uint64_t *regions,
                                 int64_t cap, uint32_t *counts, unsigned long long *below,
                                 const SelState *st, unsigned long long *ghist, uint32_t *bpart,
                                 double *dbg_out, const uint32_t *xk, hipStream_t stream)
{
    return launch_pair_tiles_t<float>(KP, mode, grid, xc, nrm, n, nb, t0, t1, regions, cap,
                                      counts, below, st, ghist, bpart, dbg_out, stream, nullptr, xk);
}

hipError_t launch_sample_tiles(int KP, const double *xc, const double *nrm, const float *xcf,
                               const float *nrmf, const uint32_t *xk, int64_t n, int64_t ntiles,
                               uint64_t *keys, hipStream_t stream)
{
    if (n / TB < 2 || ntiles <= 0) return hipErrorInvalidValue;
    const int grid = (int)(ntiles < 1024 ? ntiles : 1024);
    if (xcf)
        return launch_pair_tiles_t<float>(KP, 3, grid, xcf, nrmf, n, 0, 0, ntiles, nullptr, 0,
                                          nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                          stream, keys, xk);
    return launch_pair_tiles_t<double>(KP, 3, grid, xc, nrm, n, 0, 0, ntiles, nullptr, 0, nullptr,
                                       nullptr, nullptr, nullptr, nullptr, nullptr, stream, keys);
}

hipError_t launch_swz_f32(const double *x, int KP, const double *V, int VW, const double *cvec,
                          int64_t ntiles, float *XS, float *VS, hipStream_t stream)
{
    if (KP % 16 || VW % 16 || ntiles <= 0) return hipErrorInvalidValue;
    const int64_t tot = ntiles * TBJ * KP + ntiles * 2 * (VW / 16 + 1) * 256;
    int64_t g = (tot + 255) / 256;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_swz_f32, dim3(g), dim3(256), 0, stream, x, KP, V, VW, cvec, ntiles, XS, VS);
    return hipGetLastError();
}

#define SVGD_PHIS_CASE(KPv, NCBv)                                                            \
    if (KP == KPv && NCB == NCBv) {                                                          \
        hipLaunchKernelGGL((k_phi_f32s<KPv, NCBv>), dim3(grid), dim3(256), 0, stream, XS, VS, xrow, \
                           crow, a_ptr, row0, nrows, ntiles, d, inv_n, wv, xc, xc_stride, phi, \
                           opt ? *opt : OptArgs{}, opt ? 1 : 0);                            \
        return hipGetLastError();                                                            \
    }

bool phi_f32s_supported(int KP, int NCB) { return KP % 16 == 0 && KP <= 64 && NCB >= 1 && NCB <= 5; }

hipError_t launch_phi_f32s(int KP, int NCB, const float *XS, const float *VS, const float *xrow,
                           const float *crow, const double *a_ptr, int64_t row0, int64_t nrows,
                           int64_t ntiles, int d, double inv_n, const double *wv, const double *xc,
                           int xc_stride, double *phi, const OptArgs *opt, hipStream_t stream)
{
    if (nrows <= 0) return hipSuccess;
    if (row0 % 16) return hipErrorInvalidValue; // (waves own 16-row groups of the padded rows)
    const int64_t grid = (nrows + 63) / 64;
    SVGD_PHIS_CASE(16, 1) SVGD_PHIS_CASE(16, 2)
    SVGD_PHIS_CASE(32, 1) SVGD_PHIS_CASE(32, 2) SVGD_PHIS_CASE(32, 3)
    SVGD_PHIS_CASE(64, 1) SVGD_PHIS_CASE(64, 2) SVGD_PHIS_CASE(64, 3) SVGD_PHIS_CASE(64, 4)
    SVGD_PHIS_CASE(64, 5)
    return hipErrorInvalidValue;
}
#undef SVGD_PHIS_CASE

bool phi_b3_supported(int KP, int NCB) { return (KP == 32 || KP == 64) && NCB >= 1 && NCB <= 5; }
int64_t phi_b3_tile_words(int KP, int NCB) { return (int64_t)(6 * (KP / 32) + 3 * NCB + 2) * 256; }

int64_t median_key_part_words(int KP, int64_t np) { return kb3_keys(KP) ? (np / 16) * kb3_block_words(KP) : 0; }

hipError_t launch_swz_keys_b3(const float *xcf, int KP, int64_t np, uint32_t *XK, hipStream_t stream)
{
    if (!kb3_keys(KP) || np % 16 || np <= 0) return hipErrorInvalidValue;
    const int64_t tot = (np / 16) * (KP / 32) * 64;
    int64_t g = (tot + 255) / 256;
    if (g > 8192) g = 8192;
    if (KP == 32)
        hipLaunchKernelGGL(k_swz_keys_b3<32>, dim3(g), dim3(256), 0, stream, xcf, np / 16, XK);
    else
        hipLaunchKernelGGL(k_swz_keys_b3<64>, dim3(g), dim3(256), 0, stream, xcf, np / 16, XK);
    return hipGetLastError();
}

hipError_t launch_swz_b3(const double *x, int KP, const double *V, int VW, const double *cvec,
                         int64_t n, int64_t ntiles, uint32_t *B3, hipStream_t stream)
{
    if (!phi_b3_supported(KP, VW / 16) || VW % 16 || ntiles <= 0) return hipErrorInvalidValue;
    const int64_t tot = ntiles * (2 * (KP / 32) + VW / 16) * 64 + ntiles * 128;
    int64_t g = (tot + 255) / 256;
    if (g > 8192) g = 8192;
    if (KP == 32)
        hipLaunchKernelGGL(k_swz_b3<32>, dim3(g), dim3(256), 0, stream, x, V, VW, cvec, n, ntiles, B3);
    else
        hipLaunchKernelGGL(k_swz_b3<64>, dim3(g), dim3(256), 0, stream, x, V, VW, cvec, n, ntiles, B3);
    return hipGetLastError();
}

#ifndef SVGD_B3_NW
#define SVGD_B3_NW 8
#endif
#define SVGD_PHIB3_LAUNCH(KPv, NCBv, S1Vv, RGv)                                               \
    hipLaunchKernelGGL((k_phi_b3<KPv, NCBv, SVGD_B3_NW, S1Vv, RGv>),                            \
                       dim3((nrows + 16 * RGv * SVGD_B3_NW - 1) / (16 * RGv * SVGD_B3_NW)),     \
                       dim3(64 * SVGD_B3_NW), 0, stream, B3, crow, a_ptr, row0, nrows, ntiles, d, \
                       inv_n, wv, xc, xc_stride, phi, opt ? *opt : OptArgs{}, opt ? 1 : 0)
#define SVGD_PHIB3_CASE(KPv, NCBv)                                                           \
    if (KP == KPv && NCB == NCBv) {                                                          \
        if (d == 16 * NCBv && rg2)                                                            \
            SVGD_PHIB3_LAUNCH(KPv, NCBv, true, 2);                                            \
        else if (d == 16 * NCBv)                                                              \
            SVGD_PHIB3_LAUNCH(KPv, NCBv, true, 1);                                            \
        else if (rg2)                                                                         \
            SVGD_PHIB3_LAUNCH(KPv, NCBv, false, 2);                                           \
        else                                                                                  \
            SVGD_PHIB3_LAUNCH(KPv, NCBv, false, 1);                                           \
        return hipGetLastError();                                                            \
    }
int phi_b3_rows_per_wg(int rg) { return 16 * rg * SVGD_B3_NW; }
hipError_t launch_phi_b3(int KP, int NCB, const uint32_t *B3, const float *crow,
                         const double *a_ptr, int64_t row0, int64_t nrows, int64_t ntiles, int d,
                         double inv_n, const double *wv, const double *xc, int xc_stride,
                         double *phi, const OptArgs *opt, int rg, hipStream_t stream)
{
    if (nrows <= 0) return hipSuccess;
    if (row0 % 16) return hipErrorInvalidValue; // (waves own 16-row groups of the padded rows)
    const bool rg2 = rg == 2;
    SVGD_PHIB3_CASE(32, 1) SVGD_PHIB3_CASE(32, 2) SVGD_PHIB3_CASE(32, 3)
    SVGD_PHIB3_CASE(64, 1) SVGD_PHIB3_CASE(64, 2) SVGD_PHIB3_CASE(64, 3) SVGD_PHIB3_CASE(64, 4)
    SVGD_PHIB3_CASE(64, 5)
    return hipErrorInvalidValue;
}
#undef SVGD_PHIB3_CASE
#undef SVGD_PHIB3_LAUNCH

// fp32 norms for the tile-path median passes: rows [n, np) get +inf, so a
// padding particle's v = fma(2, dot, -n_i - n_j) is -inf (never below, never
// a candidate) without a mask in k_pair_tcol3
__global__ void k_cvt_nrm_f32(const double *__restrict__ src, int64_t n, int64_t np, float *__restrict__ dst)
{
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < np; e += (int64_t)gridDim.x * blockDim.x)
        dst[e] = e < n ? (float)src[e] : __builtin_inff();
}

hipError_t launch_cvt_nrm_f32(const double *src, int64_t n, int64_t np, float *dst, hipStream_t stream)
{
    if (np <= 0) return hipSuccess;
    int64_t g = (np + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_cvt_nrm_f32, dim3(g), dim3(256), 0, stream, src, n, np, dst);
    return hipGetLastError();
}

hipError_t launch_cvt_f32(const double *src, int64_t cnt, float *dst, hipStream_t stream)
{
    if (cnt <= 0) return hipSuccess;
    int64_t g = (cnt + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_cvt_f32, dim3(g), dim3(256), 0, stream, src, cnt, dst);
    return hipGetLastError();
}

int center_fold_grid(int d, int64_t np)
{
    int64_t g = (np + 255) / 256;
    return (int)std::min<int64_t>(g, 4096 / std::max(1, d));
}

hipError_t launch_mean_center(const double *X, int64_t n, int d, int KP, int64_t np,
                              double *partial, int nparts, double *xc, double *nrm,
                              int nrm_in_slot, float *xf, unsigned long long *nmax_bits,
                              unsigned long long *bzero, hipStream_t stream, SelState *st_out,
                              const SelState *st_init, const double *pin, int nin, double *pout,
                              unsigned long long *nmax_zero, float *xcf, float *nrmf, uint32_t *xsplit)
{
    const SelState sinit = st_init ? *st_init : SelState{};
    if (!st_init) st_out = nullptr;
    // pin: the column partials of another X (the fold, k_center_d only), else
    // the exact mean of this X from k_mean_partial's (which also zeroes
    // nmax_bits, the max target of this centring)
    const bool fold = pin && d <= 16 && KP == med_rec_stride(d);
    if (!fold) {
        hipLaunchKernelGGL(k_mean_partial, dim3(nparts), dim3(256), 0, stream, X, n, d, partial,
                           xf ? nmax_bits : nullptr);
        pin = partial;
        nin = nparts;
    }
    int64_t g = (np + 255) / 256;
    if (g > 4096) g = 4096;
    const int gd = center_fold_grid(d, np);
#define SVGD_CENTER_CASE(Dv)                                                                  \
    case Dv:                                                                                  \
        hipLaunchKernelGGL((k_center_d<Dv>), dim3(gd), dim3(256), 0, stream, X, n, pin, nin,   \
                           np, xc, nrm, nrm_in_slot, xf, nmax_bits, nmax_zero, pout, bzero, st_out, \
                           sinit, reinterpret_cast<uint4 *>(xsplit));                          \
        return hipGetLastError();
    if (d <= 16 && KP == med_rec_stride(d)) {
        switch (d) {
            SVGD_CENTER_CASE(1) SVGD_CENTER_CASE(2) SVGD_CENTER_CASE(3) SVGD_CENTER_CASE(4)
            SVGD_CENTER_CASE(5) SVGD_CENTER_CASE(6) SVGD_CENTER_CASE(7) SVGD_CENTER_CASE(8)
            SVGD_CENTER_CASE(9) SVGD_CENTER_CASE(10) SVGD_CENTER_CASE(11) SVGD_CENTER_CASE(12)
            SVGD_CENTER_CASE(13) SVGD_CENTER_CASE(14) SVGD_CENTER_CASE(15) SVGD_CENTER_CASE(16)
        default:
            break;
        }
    }
#undef SVGD_CENTER_CASE
    if (xsplit) return hipErrorInvalidValue; // (the split: k_center_d, d <= 8, only)
    if (!xf && !nrm_in_slot && (KP == 32 || KP == 64) && d <= KP && np % 2 == 0) {
        if (KP == 32)
            hipLaunchKernelGGL((k_center_t<32>), dim3(g), dim3(256), 0, stream, X, n, d, partial, nparts, np,
                               xc, nrm, xcf, nrmf, bzero, st_out, sinit);
        else
            hipLaunchKernelGGL((k_center_t<64>), dim3(g), dim3(256), 0, stream, X, n, d, partial, nparts, np,
                               xc, nrm, xcf, nrmf, bzero, st_out, sinit);
        return hipGetLastError();
    }
    if (xcf) return hipErrorInvalidValue; // (the fp32 copies: KP 32 / 64 only)
    hipLaunchKernelGGL(k_center, dim3(g), dim3(256), 0, stream, X, n, d, KP, partial, nparts, np,
                       xc, nrm, nrm_in_slot, xf, med_f32_stride(d), nmax_bits, bzero, st_out, sinit);
    return hipGetLastError();
}

hipError_t launch_prep_v(const double *xc, const double *G, const double *nrm, const double *a_ptr,
                         int64_t n, int64_t np, int d, int KP, int VW, double *V, double *cvec,
                         hipStream_t stream)
{
    int64_t g = (np * VW + 255) / 256;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_prep_v, dim3(g), dim3(256), 0, stream, xc, G, nrm, a_ptr, n, np, d, KP,
                       VW, V, cvec);
    return hipGetLastError();
}

hipError_t launch_opt_update(const OptArgs &o, const double *g, hipStream_t stream)
{
    if (o.cnt <= 0) return hipSuccess;
    int64_t grid = (o.cnt + 255) / 256;
    if (grid > 8192) grid = 8192;
    hipLaunchKernelGGL(k_opt_update, dim3(grid), dim3(256), 0, stream, o, g);
    return hipGetLastError();
}

#define SVGD_SAMPLE_CASE(Dv)                                                                 \
    case Dv:                                                                                 \
        hipLaunchKernelGGL((k_sample_keys_f32<Dv>), dim3(g), dim3(256), 0, stream, xf, n, g0, S, keys, \
                           init, st_out);                                                    \
        break;

hipError_t launch_sample_keys(const double *xc, const double *nrm, const float *xf, int64_t n,
                              int d, int KP, int64_t g0, int64_t S, uint64_t *keys,
                              const SelState &init, SelState *st_out, hipStream_t stream)
{
    int64_t g = (S + 255) / 256;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1; // (writes st_out even for an empty sample shard)
    if (!xf) {
        hipLaunchKernelGGL(k_sample_keys, dim3(g), dim3(256), 0, stream, xc, nrm, n, d, KP, g0, S,
                           keys, init, st_out);
        return hipGetLastError();
    }
    switch (d) {
        SVGD_SAMPLE_CASE(1) SVGD_SAMPLE_CASE(2) SVGD_SAMPLE_CASE(3) SVGD_SAMPLE_CASE(4)
        SVGD_SAMPLE_CASE(5) SVGD_SAMPLE_CASE(6) SVGD_SAMPLE_CASE(7) SVGD_SAMPLE_CASE(8)
        SVGD_SAMPLE_CASE(9) SVGD_SAMPLE_CASE(10) SVGD_SAMPLE_CASE(11) SVGD_SAMPLE_CASE(12)
        SVGD_SAMPLE_CASE(13) SVGD_SAMPLE_CASE(14) SVGD_SAMPLE_CASE(15) SVGD_SAMPLE_CASE(16)
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_hist_regions(const uint64_t *keys, const uint32_t *counts, int64_t nreg,
                               int64_t cap, int max_blocks, const SelState *st,
                               unsigned long long *ghist, hipStream_t stream)
{
    if (nreg <= 0) return hipSuccess;
    int64_t G = HIST_BLOCKS;
    if (max_blocks > 0 && G > max_blocks) G = max_blocks;
    if (nreg < G) G = (G / nreg) * nreg; // whole slices per region
    if (G < 1) G = 1;
    hipLaunchKernelGGL(k_hist_regions, dim3(G), dim3(256), 0, stream, keys, counts, nreg, cap, st,
                       ghist);
    return hipGetLastError();
}

hipError_t launch_compact(const uint64_t *keys, const uint32_t *counts, int64_t nreg, int64_t cap,
                          const SelState *st, uint64_t *cbuf, unsigned long long *ccount,
                          hipStream_t stream)
{
    if (nreg <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(ccount, 0, sizeof(unsigned long long), stream);
    if (e != hipSuccess) return e;
    const int64_t G = nreg < 8192 ? nreg : 8192;
    hipLaunchKernelGGL(k_compact, dim3(G), dim3(256), 0, stream, keys, counts, nreg, cap, st, cbuf,
                       ccount);
    return hipGetLastError();
}

hipError_t launch_select_tail(SelState *st, const uint64_t *cbuf, const unsigned long long *ccount,
                              int passes, hipStream_t stream)
{
    if (passes <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_select_tail, dim3(1), dim3(1024), 0, stream, st, cbuf, ccount, passes);
    return hipGetLastError();
}

hipError_t launch_hist_count(const uint64_t *keys, const unsigned long long *ccount, int64_t cap,
                             const SelState *st, unsigned long long *ghist, hipStream_t stream)
{
    // one region whose count lives on the device (compacted keys; < 2^32)
    return launch_hist_regions(keys, reinterpret_cast<const uint32_t *>(ccount), 1, cap, 64, st,
                               ghist, stream);
}

hipError_t launch_select_scan(SelState *st, unsigned long long *ghist, int make_bracket,
                              unsigned long long *bzero, hipStream_t stream)
{
    hipLaunchKernelGGL(k_select_scan, dim3(1), dim3(256), 0, stream, st, ghist, make_bracket, bzero);
    return hipGetLastError();
}

hipError_t launch_counts_reduce(const unsigned long long *below, const uint32_t *counts,
                                int64_t nblk, int64_t cap, const SelState *st,
                                const uint32_t *bpart, int64_t nbpart,
                                unsigned long long *cnt, hipStream_t stream, uint64_t *seg_zero)
{
    hipLaunchKernelGGL(k_counts_reduce, dim3(NBK / 64 * BSUM_SLICES + 1), dim3(256), 0, stream, below,
                       counts, nblk, cap, st, bpart, nbpart, cnt, seg_zero);
    return hipGetLastError();
}

hipError_t launch_set_state(const SelState &s, SelState *st, hipStream_t stream)
{
    hipLaunchKernelGGL(k_set_state, dim3(1), dim3(1), 0, stream, s, st);
    return hipGetLastError();
}

hipError_t launch_set_scal(double a, double med, double *scal, hipStream_t stream)
{
    hipLaunchKernelGGL(k_set_scal, dim3(1), dim3(1), 0, stream, a, med, scal);
    return hipGetLastError();
}

hipError_t launch_set_sel(SelState *st, int nsel, uint64_t r0, uint64_t r1, int b0, int b1,
                          uint64_t *seg, hipStream_t stream)
{
    hipLaunchKernelGGL(k_set_sel, dim3(1), dim3(1), 0, stream, st, nsel, r0, r1, b0, b1, seg);
    return hipGetLastError();
}

hipError_t launch_compact_buckets(const uint64_t *keys, const uint32_t *counts, int64_t nreg,
                                  int64_t cap, SelState *st, uint64_t *seg, int64_t seg_cap,
                                  const int *status, hipStream_t stream, const PlanArgs *plan)
{
    if (nreg <= 0 && !plan) return hipSuccess;
    int64_t G = (nreg + 3) / 4; // one region per wave
    if (G > 512) G = 512;
    if (G < 1) G = 1; // (with a plan the launch publishes it even without regions)
    hipLaunchKernelGGL(k_compact_buckets, dim3(G), dim3(256), 0, stream, keys, counts, nreg, cap,
                       st, seg, seg_cap, status, plan ? *plan : PlanArgs{});
    return hipGetLastError();
}

hipError_t launch_select_small(SelState *st, const uint64_t *segs, int nseg, int64_t seg_cap,
                               int navg, int src_lo, int src_hi, double logn, double *scal,
                               const int *status, hipStream_t stream, uint64_t *trk, uint64_t seq)
{
    hipLaunchKernelGGL(k_select_small, dim3(1), dim3(1024), 0, stream, st, segs, nseg, seg_cap,
                       navg, src_lo, src_hi, logn, scal, status, trk, seq);
    return hipGetLastError();
}

hipError_t launch_plan_select(const unsigned long long *cnt, SelState *st, int nsel, uint64_t r0,
                              uint64_t r1, int64_t capr, uint64_t *seg, int *status,
                              int *host_status, hipStream_t stream)
{
    hipLaunchKernelGGL(k_plan_select, dim3(1), dim3(256), 0, stream, cnt, st, nsel, r0, r1, capr,
                       seg, status, host_status);
    return hipGetLastError();
}

hipError_t launch_scale_factor(const double *src, double factor, int d, double *M, double *L,
                               double *sgn, double *work, double *scal, int *err, hipStream_t stream)
{
    hipLaunchKernelGGL(k_scale_factor, dim3(1), dim3(64), 0, stream, src, factor, d, M, L, sgn, work,
                       scal, err);
    return hipGetLastError();
}

hipError_t launch_prep_rec_mat(const double *xc, const double *G, const double *M, const double *L,
                               const double *sgn, int64_t n, int64_t np, int d, int KP, int RS,
                               double *rec, double *wv, hipStream_t stream)
{
    int64_t g = (np + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_prep_rec_mat, dim3(g), dim3(256), 0, stream, xc, G, M, L, sgn, n, np, d, KP,
                       RS, rec, wv);
    return hipGetLastError();
}

hipError_t launch_prep_v_mat(const double *xc, const double *G, const double *M, const double *L,
                             int64_t n, int64_t np, int d, int KP, int VW, double *zc, double *V,
                             double *cvec, double *wv, hipStream_t stream)
{
    int64_t g = (np + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_prep_v_mat, dim3(g), dim3(256), 0, stream, xc, G, M, L, n, np, d, KP, VW,
                       zc, V, cvec, wv);
    return hipGetLastError();
}

hipError_t launch_gauss_grad(const double *X, int64_t rows, int d, int k, const double *mu,
                             const double *prec, double *G, hipStream_t stream)
{
    if (rows <= 0) return hipSuccess;
    const int64_t g = (rows + 255) / 256;
#define SVGD_GG_CASE(Dv)                                                                     \
    case Dv:                                                                                 \
        hipLaunchKernelGGL((k_gauss_grad<Dv>), dim3(g), dim3(256), 0, stream, X, rows, d, k, mu, \
                           prec, G);                                                         \
        break;
    switch (d) {
        SVGD_GG_CASE(1) SVGD_GG_CASE(2) SVGD_GG_CASE(3) SVGD_GG_CASE(4)
        SVGD_GG_CASE(5) SVGD_GG_CASE(6) SVGD_GG_CASE(7) SVGD_GG_CASE(8)
        SVGD_GG_CASE(12) SVGD_GG_CASE(16)
    default:
        if (d > 64) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_gauss_grad<0>), dim3(g), dim3(256), 0, stream, X, rows, d, k, mu,
                           prec, G);
    }
#undef SVGD_GG_CASE
    return hipGetLastError();
}

hipError_t launch_finalize(const SelState *st, int navg, int src_lo, int src_hi, double logn,
                           double *a_out, double *med_out, hipStream_t stream)
{
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(1), 0, stream, st, navg, src_lo, src_hi, logn,
                       a_out, med_out);
    return hipGetLastError();
}

} // namespace svgd_amd

namespace svgd_amd {

bool phi_sym_supported(int d) { return d >= 1 && d <= 8; }

#define SVGD_SYM_GEOM(Dv)                                                                    \
    case Dv:                                                                                 \
        *B = SymGeom<Dv>::B;                                                                 \
        *SRS = SymGeom<Dv>::SRS;                                                             \
        *NSUB = SymGeom<Dv>::NSUB;                                                           \
        return true;
bool phi_sym_geom(int d, int *B, int *SRS, int *NSUB)
{
    switch (d) {
        SVGD_SYM_GEOM(1) SVGD_SYM_GEOM(2) SVGD_SYM_GEOM(3) SVGD_SYM_GEOM(4)
        SVGD_SYM_GEOM(5) SVGD_SYM_GEOM(6) SVGD_SYM_GEOM(7) SVGD_SYM_GEOM(8)
    default:
        return false;
    }
}

int phi_sym_blocks_per_cu(int d)
{
    int nb = 0;
    hipError_t e = hipErrorInvalidValue;
    switch (d) {
    case 1: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_phi_sym<1>, SYM_NW * 64, 0); break;
    case 2: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_phi_sym<2>, SYM_NW * 64, 0); break;
    case 3: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_phi_sym<3>, SYM_NW * 64, 0); break;
    case 4: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_phi_sym<4>, SYM_NW * 64, 0); break;
    case 5: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_phi_sym<5>, SYM_NW * 64, 0); break;
    case 6: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_phi_sym<6>, SYM_NW * 64, 0); break;
    case 7: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_phi_sym<7>, SYM_NW * 64, 0); break;
    case 8: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_phi_sym<8>, SYM_NW * 64, 0); break;
    default: break;
    }
    return (e == hipSuccess && nb > 0) ? nb : 1;
}

#define SVGD_SYM_CASE(Dv)                                                                     \
    case Dv: {                                                                                \
        using Gm = SymGeom<Dv>;                                                               \
        const int64_t npad = a.nbs * Gm::B;                                                   \
        int64_t g = (npad + 255) / 256;                                                       \
        if (g > 4096) g = 4096;                                                               \
        hipLaunchKernelGGL((k_prep_sym<Dv>), dim3(g), dim3(256), 0, stream, a.xc, a.KP, a.G,   \
                           a.nrm, a.a_ptr, a.nmax, a.n, npad, a.srec, a.symok, a.rec, a.RS);  \
        if ((e = hipGetLastError()) != hipSuccess) return e;                                  \
        if (ev_k0 && (e = hipEventRecord(ev_k0, stream)) != hipSuccess) return e;             \
        const SymRows fr{a.rec, a.row0, a.nrows, a.n, a.fS,                                   \
                         ((a.nrows + phi_rows_t8k_rows(4) - 1) / phi_rows_t8k_rows(4)) * a.fS,  \
                         a.fpart, a.fldp, a.nmax};                                            \
        hipLaunchKernelGGL((k_phi_sym<Dv>), dim3(a.grid), dim3(SYM_NW * 64), 0, stream, a.srec, a.a_ptr, \
                           a.nbs, a.u0, a.u1, a.symok, a.rowpart, a.blkg, a.rbase, a.colpart, a.SM, \
                           a.wst, a.qlast, a.tab8k, fr);                                      \
        if ((e = hipGetLastError()) != hipSuccess) return e;                                  \
        if (ev_k1 && (e = hipEventRecord(ev_k1, stream)) != hipSuccess) return e;             \
        return hipSuccess;                                                                    \
    }

#define SVGD_SYM_FINISH_CASE(Dv)                                                              \
    case Dv: {                                                                                \
        constexpr int RB = 256 / SymGeom<Dv>::DP;                                             \
        /* P > 1 (contrib): only the particles this rank's units touch -- the    \
           row blocks Ia .. Ib and up to SM - 1 blocks ahead, a cyclic run;      \
           the others' sums stay zero from the allocation and are never sent */  \
        const int64_t B_ = SymGeom<Dv>::B;                                                    \
        const int64_t fr0 = a.contrib ? a.Ia * B_ : a.row0;                                   \
        const int64_t fn = a.contrib ? std::min<int64_t>(a.n, (a.Ib - a.Ia + a.SM) * B_) : a.nrows; \
        if (fn <= 0) return hipSuccess;                                                       \
        hipLaunchKernelGGL((k_sym_finish<Dv>), dim3((fn + RB - 1) / RB), dim3(256), 0,         \
                           stream, a.rowpart, a.colpart, a.srec, a.a_ptr, a.nbs, a.SM, a.Ia,   \
                           a.Ib, a.blkg, a.rbase, a.symok, fr0, fn, a.inv_n, a.phi,            \
                           opt ? *opt : OptArgs{}, opt ? 1 : 0, a.contrib,                    \
                           a.contrib ? a.n : (int64_t)0, fb);                                 \
        return hipGetLastError();                                                             \
    }

#define SVGD_SYM_APPLY_CASE(Dv)                                                               \
    case Dv: {                                                                                \
        constexpr int RB = 256 / SymGeom<Dv>::DP;                                             \
        hipLaunchKernelGGL((k_sym_apply<Dv>), dim3((a.nrows + RB - 1) / RB), dim3(256), 0,     \
                           stream, own, recv, xtab, world, rank, a.srec, a.a_ptr, a.symok,     \
                           a.row0, a.nrows, a.inv_n,                                           \
                           a.phi, opt ? *opt : OptArgs{}, opt ? 1 : 0, fb);                   \
        return hipGetLastError();                                                             \
    }

static SymFallback sym_fallback(const SymArgs &a)
{
    return SymFallback{a.fpart, a.fS, a.fldp, a.rec, a.RS};
}

hipError_t launch_sym_apply(const SymArgs &a, const double *own, const double *recv, const int64_t *xtab,
                            int world, int rank, const OptArgs *opt, hipStream_t stream)
{
    if (world > 1 && !xtab) return hipErrorInvalidValue;
    if (a.nrows <= 0) return hipSuccess;
    const SymFallback fb = sym_fallback(a);
    switch (a.d) {
        SVGD_SYM_APPLY_CASE(1) SVGD_SYM_APPLY_CASE(2) SVGD_SYM_APPLY_CASE(3) SVGD_SYM_APPLY_CASE(4)
        SVGD_SYM_APPLY_CASE(5) SVGD_SYM_APPLY_CASE(6) SVGD_SYM_APPLY_CASE(7) SVGD_SYM_APPLY_CASE(8)
    default:
        return hipErrorInvalidValue;
    }
}

hipError_t launch_sym_finish(const SymArgs &a, const OptArgs *opt, hipStream_t stream)
{
    const SymFallback fb = sym_fallback(a);
    switch (a.d) {
        SVGD_SYM_FINISH_CASE(1) SVGD_SYM_FINISH_CASE(2) SVGD_SYM_FINISH_CASE(3) SVGD_SYM_FINISH_CASE(4)
        SVGD_SYM_FINISH_CASE(5) SVGD_SYM_FINISH_CASE(6) SVGD_SYM_FINISH_CASE(7) SVGD_SYM_FINISH_CASE(8)
    default:
        return hipErrorInvalidValue;
    }
}

hipError_t launch_phi_sym(const SymArgs &a, hipEvent_t ev_k0, hipEvent_t ev_k1, hipStream_t stream)
{
    hipError_t e = hipSuccess;
    if (a.nrows <= 0 && !a.contrib) return hipSuccess; // (P > 1: the rank's units still count)
    switch (a.d) {
        SVGD_SYM_CASE(1) SVGD_SYM_CASE(2) SVGD_SYM_CASE(3) SVGD_SYM_CASE(4)
        SVGD_SYM_CASE(5) SVGD_SYM_CASE(6) SVGD_SYM_CASE(7) SVGD_SYM_CASE(8)
    default:
        return hipErrorInvalidValue;
    }
}

#define SVGD_OCC_CASE(Dv)                                                                    \
    case Dv:                                                                                 \
        e = R == 1   ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_phi_rows<Dv, 1>, 256, 0) \
            : R == 2 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_phi_rows<Dv, 2>, 256, 0) \
                     : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_phi_rows<Dv, 4>, 256, 0); \
        break;

int phi_rows_blocks_per_cu(int d, int R, int kind)
{
    int nb = 0;
    hipError_t e = hipErrorInvalidValue;
    if (kind == 2) {
#define SVGD_T8K_OCC(Dv)                                                                          \
    case Dv:                                                                                      \
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, SVGD_T8K_KERNEL(Dv), T8K_NW * 64, 0); \
        break;
        switch (d) {
            SVGD_T8K_OCC(1) SVGD_T8K_OCC(2) SVGD_T8K_OCC(3) SVGD_T8K_OCC(4)
            SVGD_T8K_OCC(5) SVGD_T8K_OCC(6) SVGD_T8K_OCC(7) SVGD_T8K_OCC(8)
            SVGD_T8K_OCC(9) SVGD_T8K_OCC(10) SVGD_T8K_OCC(11) SVGD_T8K_OCC(12)
            SVGD_T8K_OCC(13) SVGD_T8K_OCC(14) SVGD_T8K_OCC(15) SVGD_T8K_OCC(16)
        default:
            break;
        }
#undef SVGD_T8K_OCC
        return (e == hipSuccess && nb > 0) ? nb : 1;
    }
    switch (d) {
        SVGD_OCC_CASE(1) SVGD_OCC_CASE(2) SVGD_OCC_CASE(3) SVGD_OCC_CASE(4)
        SVGD_OCC_CASE(5) SVGD_OCC_CASE(6) SVGD_OCC_CASE(7) SVGD_OCC_CASE(8)
        SVGD_OCC_CASE(9) SVGD_OCC_CASE(10) SVGD_OCC_CASE(11) SVGD_OCC_CASE(12)
        SVGD_OCC_CASE(13) SVGD_OCC_CASE(14) SVGD_OCC_CASE(15) SVGD_OCC_CASE(16)
    default:
        break;
    }
    return (e == hipSuccess && nb > 0) ? nb : 1;
}

} // namespace svgd_amd

