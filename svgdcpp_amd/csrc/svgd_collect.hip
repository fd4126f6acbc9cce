// svgd_collect.hip -- the median bracket collect pass on the matrix cores
// (gfx950).  Built with VGPR-form MFMA operands (Makefile), which the other
// kernels are not.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <type_traits>

#include "svgd_device.h"

namespace svgd_amd {

typedef f4_t f4;

// ====================================== median collect on the matrix cores ==
//
// The bracket collect pass (MODE 0 of k_pair_rows) for d <= 16, fp64 keys:
// every pair is CLASSIFIED from an fp32 Gram product on v_mfma_f32_16x16x4f32
// and only the pairs whose class the fp32 value cannot decide -- the band
// around the bracket, ~0.2 % of pairs -- form their exact fp64 key, with the
// same arithmetic as k_pair_rows / k_sample_keys (so every pass still agrees
// bit for bit).  GaussianRBFKernel.hpp:179-187 (the pairwise distances whose
// median is taken).
//
// MFMA roles: A = 16 columns j (lane l: x_j[j0 + l%16][4kk + l/16]), B = 16
// rows i (same pattern), C = h_j = -|x_j|^2/2 of the lane's output rows, so
// lane l holds ef = h_j + x_i.x_j for i = i0 + l%16, j = j0 + 4(l/16) + r.
//
// Error bound (u = 2^-24, MFMA f32 == an fmaf chain, MI355X_MICROARCH.md):
// inputs rounded to fp32 (u each), products exact in the fma, D roundings of
// the partial sums, so |ef - e| <= 1.01 (D + 3) u S with S = |h_j| +
// sum_k |x_ik x_jk| <= 1.5 nmax.  MCOL_DELTA(D) = 4 (D + 4) u nmax (> 2.6x
// that) plus 2^-100 for flushed denormals.  With the fp64 thresholds TL_i,
// TH_i of k_pair_rows (e > TL => key < lo, e <= TH => key >= hi):
//   ef >  TLf_i = up(TL_i + delta)    => below (counted)
//   ef <= THf_i = down(TH_i - delta)  => above (dropped)
// otherwise the pair is staged in LDS (one entry per lane and 16 x 16 block)
// and finished exactly
// in a batch (mcol_flush).  Data outside |x|^2 <= 2^40 sets delta = inf:
// every pair is then finished exactly (correct, slow).
constexpr int MC_STG = 256; // staged band pairs per wave
constexpr int MC_NG = 4;    // 16-row blocks per classification group
// Timing ablations of k_pair_mcol (tools/gpu_mcol_abl.sh; WRONG results, never
// a shipped build): 1 = no band staging, 2 = MFMAs only (no classification),
// 3 = staging without the exact flush
#ifndef SVGD_MCOL_ABL
#define SVGD_MCOL_ABL 0
#endif
// Band staging form: 0 = exec-masked store under a branch on "any band
// value", 1 = the same branch, every lane stores (lanes without band values,
// and entries past the area, into a 64-slot spill zone: no exec change, no
// second branch), 2 = as 1 without the branch (every block)
#ifndef SVGD_MCOL_STAGE
#define SVGD_MCOL_STAGE 1
#endif
// Off-diagonal classification form: 0 = lane masks (v_cmp into SGPRs, the
// below count and the band OR on the scalar unit), 1 = sign bits on the
// vector unit (v_pk_add_f32 of TLf - v and THf - v, a per-lane below count,
// the band as (THf - v) & ~(TLf - v): no scalar work per block), 2 = the
// band's centre and half-width (bf16-split form; the f32 form takes 0):
// mcol_classify4m, cfg3 k_pair_mcol 449 -> 428 us (profiles/r05_mcol_cls2_ab.txt)
#ifndef SVGD_MCOL_CLS
#define SVGD_MCOL_CLS 2
#endif


__device__ __forceinline__ float f32_up(double x)
{
    float f = (float)x;
    if ((double)f < x) f = f == 0.0f ? 0x1p-149f : __int_as_float(__float_as_int(f) + (f > 0.0f ? 1 : -1));
    return f;
}
__device__ __forceinline__ float f32_down(double x)
{
    float f = (float)x;
    if ((double)f > x) f = f == 0.0f ? -0x1p-149f : __int_as_float(__float_as_int(f) + (f > 0.0f ? -1 : 1));
    return f;
}

// The 4 values of one 16 x 16 block for one lane, in issue order (the
// compiler otherwise hoists every compare of a group and spills their lane
// masks): 8 compares straight into lane masks, then on the scalar unit
//   nbelow += popc(v_r > tl)          (below lo, counted)
//   h_r     = (v_r > th) & ~(v_r > tl)  (the band lanes of value r)
// so the first scalar read of a mask comes 8 vector instructions after its
// compare.  Returns h_0 | h_1 | h_2 | h_3; h_r stay in SGPRs for the staging.
// Exec is all ones here (uniform control flow); a VALU-written SGPR read by
// the SALU needs no wait states.
__device__ __forceinline__ unsigned long long mcol_classify4(const f4_t &v, float tl, float th,
                                                             uint32_t &nbelow,
                                                             unsigned long long (&h)[4])
{
    unsigned long long l0, l1, l2, l3, any;
    uint32_t t0, t1;
    asm volatile("v_cmp_gt_f32_e64 %[l0], %[v0], %[tl]\n\t"
                 "v_cmp_gt_f32_e64 %[h0], %[v0], %[th]\n\t"
                 "v_cmp_gt_f32_e64 %[l1], %[v1], %[tl]\n\t"
                 "v_cmp_gt_f32_e64 %[h1], %[v1], %[th]\n\t"
                 "v_cmp_gt_f32_e64 %[l2], %[v2], %[tl]\n\t"
                 "v_cmp_gt_f32_e64 %[h2], %[v2], %[th]\n\t"
                 "v_cmp_gt_f32_e64 %[l3], %[v3], %[tl]\n\t"
                 "v_cmp_gt_f32_e64 %[h3], %[v3], %[th]\n\t"
                 "s_bcnt1_i32_b64 %[t0], %[l0]\n\t"
                 "s_bcnt1_i32_b64 %[t1], %[l1]\n\t"
                 "s_andn2_b64 %[h0], %[h0], %[l0]\n\t"
                 "s_andn2_b64 %[h1], %[h1], %[l1]\n\t"
                 "s_add_u32 %[nb], %[nb], %[t0]\n\t"
                 "s_add_u32 %[nb], %[nb], %[t1]\n\t"
                 "s_bcnt1_i32_b64 %[t0], %[l2]\n\t"
                 "s_bcnt1_i32_b64 %[t1], %[l3]\n\t"
                 "s_andn2_b64 %[h2], %[h2], %[l2]\n\t"
                 "s_andn2_b64 %[h3], %[h3], %[l3]\n\t"
                 "s_add_u32 %[nb], %[nb], %[t0]\n\t"
                 "s_add_u32 %[nb], %[nb], %[t1]\n\t"
                 "s_or_b64 %[any], %[h0], %[h1]\n\t"
                 "s_or_b64 %[any], %[any], %[h2]\n\t"
                 "s_or_b64 %[any], %[any], %[h3]"
                 : [nb] "+s"(nbelow), [any] "=&s"(any), [l0] "=&s"(l0), [l1] "=&s"(l1),
                   [l2] "=&s"(l2), [l3] "=&s"(l3), [h0] "=&s"(h[0]), [h1] "=&s"(h[1]),
                   [h2] "=&s"(h[2]), [h3] "=&s"(h[3]), [t0] "=&s"(t0), [t1] "=&s"(t1)
                 : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [tl] "v"(tl),
                   [th] "v"(th)
                 : "scc");
    return any;
}
// SVGD_MCOL_CLS = 1: the same classes from sign bits.  For finite v and
// thresholds, fl(T - v) < 0 (sign set, -0 included) <=> v > T (a difference of
// distinct floats is never +0), T = +inf gives +inf (never), v = -inf (padding)
// gives +inf (never); so the sign of TLf - v is "below" and the sign of
// (THf - v) & ~(TLf - v) "band", as mcol_classify4's masks.  cnt += the
// lane's below values; b[r] carry the band bits in their signs.
__device__ __forceinline__ void mcol_classify4v(const f4_t &v, float tl, float th, uint32_t &cnt,
                                                uint32_t (&b)[4])
{
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 tl2 = {tl, tl}, th2 = {th, th};
    const f2 v01 = {v[0], v[1]}, v23 = {v[2], v[3]};
    const f2 a01 = tl2 - v01, a23 = tl2 - v23, t01 = th2 - v01, t23 = th2 - v23;
    const uint32_t a[4] = {__float_as_uint(a01[0]), __float_as_uint(a01[1]), __float_as_uint(a23[0]),
                           __float_as_uint(a23[1])};
    const uint32_t t[4] = {__float_as_uint(t01[0]), __float_as_uint(t01[1]), __float_as_uint(t23[0]),
                           __float_as_uint(t23[1])};
    cnt += (a[0] >> 31) + (a[1] >> 31) + (a[2] >> 31) + (a[3] >> 31);
#pragma unroll
    for (int r = 0; r < 4; ++r) b[r] = t[r] & ~a[r];
}

// SVGD_MCOL_CLS = 2: one compare per value.  Per row, with the fp32
// thresholds TL > TH of the lane-mask form clamped into [-2^42, 2^42] (every
// value is finite and below 2^41 in magnitude while delta is finite: |v| <=
// 1.5 nmax + rounding, nmax <= 2^40), TM = fp32((TL + TH) / 2) and
// W = fp32_up(max(TL - TM, TM - TH) (1 + 2^-22)), and x = fl(v - TM):
//   x > W   => v - TM > W (1 - 2^-24) >= TL - TM  => v > TL  (below)
//   x < -W  => v < TM - W (1 - 2^-24) <= TH                 (above)
// (fl(v - TM) = (v - TM)(1 + e), |e| <= 2^-24; exact when subnormal), so
// "below" is a subset of the lane-mask form's below, "above" of its above,
// and the band |x| <= W a superset of its band: the exact fp64 finish
// decides every staged pair, the keys and counts are the same.  Padding
// rows: TM = +inf, W = 0 (x is -inf or NaN: never below, never band);
// padding columns (h = -inf): x = -inf, never band.  delta = inf (nmax >
// 2^40) keeps the lane-mask form (the caller's uniform branch).
//   4 v_cmp (below) + min3 / min of |x| + 1 v_cmp (any band lane) on the
// vector unit, 4 bcnt + 4 add on the scalar unit: 8 scalar operations fewer
// per 16 x 16 block than mcol_classify4; the band lanes' per-value masks are
// formed only in the (rare) staging branch (mcol_band4m).
__device__ __forceinline__ unsigned long long mcol_classify4m(const float (&x)[4], float w, uint32_t &nbelow,
                                                              unsigned long long (&l)[4])
{
    unsigned long long &l0 = l[0], &l1 = l[1], &l2 = l[2], &l3 = l[3], any;
    uint32_t t0, t1;
    float m;
    asm volatile("v_cmp_gt_f32_e64 %[l0], %[x0], %[w]\n\t"
                 "v_cmp_gt_f32_e64 %[l1], %[x1], %[w]\n\t"
                 "v_min3_f32 %[m], |%[x0]|, |%[x1]|, |%[x2]|\n\t"
                 "v_cmp_gt_f32_e64 %[l2], %[x2], %[w]\n\t"
                 "v_cmp_gt_f32_e64 %[l3], %[x3], %[w]\n\t"
                 "v_min_f32_e64 %[m], %[m], |%[x3]|\n\t"
                 "s_bcnt1_i32_b64 %[t0], %[l0]\n\t"
                 "s_bcnt1_i32_b64 %[t1], %[l1]\n\t"
                 "v_cmp_ge_f32_e64 %[any], %[w], %[m]\n\t"
                 "s_add_u32 %[nb], %[nb], %[t0]\n\t"
                 "s_add_u32 %[nb], %[nb], %[t1]\n\t"
                 "s_bcnt1_i32_b64 %[t0], %[l2]\n\t"
                 "s_bcnt1_i32_b64 %[t1], %[l3]\n\t"
                 "s_add_u32 %[nb], %[nb], %[t0]\n\t"
                 "s_add_u32 %[nb], %[nb], %[t1]"
                 : [nb] "+s"(nbelow), [any] "=&s"(any), [l0] "=&s"(l0), [l1] "=&s"(l1),
                   [l2] "=&s"(l2), [l3] "=&s"(l3), [t0] "=&s"(t0), [t1] "=&s"(t1), [m] "=&v"(m)
                 : [x0] "v"(x[0]), [x1] "v"(x[1]), [x2] "v"(x[2]), [x3] "v"(x[3]), [w] "v"(w)
                 : "scc");
    return any;
}
// x_r = v_r - TM, two values per packed subtraction
__device__ __forceinline__ void mcol_sub_centre(const f4_t &v, float tm, float (&x)[4])
{
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 t = {tm, tm};
    const f2 x01 = f2{v[0], v[1]} - t, x23 = f2{v[2], v[3]} - t;
    x[0] = x01[0];
    x[1] = x01[1];
    x[2] = x23[0];
    x[3] = x23[1];
}
// the per-value band masks of mcol_classify4m's values (|x_r| <= W)
__device__ __forceinline__ void mcol_band4m(const float (&x)[4], float w, unsigned long long (&h)[4])
{
    asm volatile("v_cmp_ge_f32_e64 %[h0], %[w], |%[x0]|\n\t"
                 "v_cmp_ge_f32_e64 %[h1], %[w], |%[x1]|\n\t"
                 "v_cmp_ge_f32_e64 %[h2], %[w], |%[x2]|\n\t"
                 "v_cmp_ge_f32_e64 %[h3], %[w], |%[x3]|"
                 : [h0] "=&s"(h[0]), [h1] "=&s"(h[1]), [h2] "=&s"(h[2]), [h3] "=&s"(h[3])
                 : [x0] "v"(x[0]), [x1] "v"(x[1]), [x2] "v"(x[2]), [x3] "v"(x[3]), [w] "v"(w));
}
// (TM, W) of one row from the lane-mask form's fp32 thresholds (TL, TH)
__device__ __forceinline__ float2 mcol_centre_width(float tl, float th)
{
    if (tl == __builtin_inff() && th == __builtin_inff()) return make_float2(__builtin_inff(), 0.0f); // padding row
    const double L = fmin((double)tl, 0x1p42), H = fmax((double)th, -0x1p42);
    const float tm = (float)(0.5 * (L + H));
    const double w = fmax(L - (double)tm, (double)tm - H) * (1.0 + 0x1p-22);
    return make_float2(tm, f32_up(w));
}

// Diagonal tiles (1 in nb/2 of them): lanes with xl > c (j > i) only.
// Returns the band lanes of the value.
__device__ __forceinline__ unsigned long long mcol_classify_diag(float v, float tl, float th, int xl,
                                                                 int c, uint32_t &nbelow)
{
    unsigned long long ml, mh, ok;
    uint32_t t;
    asm volatile("v_cmp_gt_i32_e64 %[ok], %[xl], %[c]\n\t"
                 "v_cmp_gt_f32_e64 %[ml], %[v], %[tl]\n\t"
                 "v_cmp_gt_f32_e64 %[mh], %[v], %[th]\n\t"
                 "s_and_b64 %[ml], %[ml], %[ok]\n\t"
                 "s_and_b64 %[mh], %[mh], %[ok]\n\t"
                 "s_bcnt1_i32_b64 %[t], %[ml]\n\t"
                 "s_add_u32 %[nb], %[nb], %[t]\n\t"
                 "s_andn2_b64 %[mh], %[mh], %[ml]"
                 : [nb] "+s"(nbelow), [ml] "=&s"(ml), [mh] "=&s"(mh), [ok] "=&s"(ok), [t] "=&s"(t)
                 : [v] "v"(v), [tl] "v"(tl), [th] "v"(th), [xl] "v"(xl), [c] "s"(c)
                 : "scc");
    return mh;
}

// Diagonal tiles in the centre form (x = v - TM, half-width W; as
// mcol_classify4m): below (x > W) and band (|x| <= W) lanes among those with
// xl > c (j > i).  Returns the band lanes of the value.
__device__ __forceinline__ unsigned long long mcol_classify_diag_m(float x, float w, int xl, int c,
                                                                   uint32_t &nbelow)
{
    unsigned long long ml, mb, ok;
    uint32_t t;
    asm volatile("v_cmp_gt_i32_e64 %[ok], %[xl], %[c]\n\t"
                 "v_cmp_gt_f32_e64 %[ml], %[x], %[w]\n\t"
                 "v_cmp_ge_f32_e64 %[mb], %[w], |%[x]|\n\t"
                 "s_and_b64 %[ml], %[ml], %[ok]\n\t"
                 "s_and_b64 %[mb], %[mb], %[ok]\n\t"
                 "s_bcnt1_i32_b64 %[t], %[ml]\n\t"
                 "s_add_u32 %[nb], %[nb], %[t]"
                 : [nb] "+s"(nbelow), [ml] "=&s"(ml), [mb] "=&s"(mb), [ok] "=&s"(ok), [t] "=&s"(t)
                 : [x] "v"(x), [w] "v"(w), [xl] "v"(xl), [c] "s"(c)
                 : "scc");
    return mb;
}

// The lane's bits of the 4 band masks of one 16 x 16 block (bit r: value r
// is a band value), straight from the scalar masks.
__device__ __forceinline__ uint32_t mcol_code4(const unsigned long long (&h)[4])
{
    uint32_t c0, c1, c2, c3;
    asm volatile("v_cndmask_b32_e64 %[c0], 0, 1, %[h0]\n\t"
                 "v_cndmask_b32_e64 %[c1], 0, 2, %[h1]\n\t"
                 "v_cndmask_b32_e64 %[c2], 0, 4, %[h2]\n\t"
                 "v_cndmask_b32_e64 %[c3], 0, 8, %[h3]"
                 : [c0] "=&v"(c0), [c1] "=&v"(c1), [c2] "=&v"(c2), [c3] "=&v"(c3)
                 : [h0] "s"(h[0]), [h1] "s"(h[1]), [h2] "s"(h[2]), [h3] "s"(h[3]));
    return c0 | c1 | c2 | c3;
}

// a (lanes in mask) or b (the others), straight from a scalar lane mask
__device__ __forceinline__ uint32_t mcol_sel(unsigned long long mask, uint32_t a, uint32_t b)
{
    uint32_t r;
    asm volatile("v_cndmask_b32_e64 %[r], %[b], %[a], %[m]" : [r] "=v"(r) : [a] "v"(a), [b] "v"(b), [m] "s"(mask));
    return r;
}

// Row operands of one 16-row block for one lane: B (KK fp32) | TLf | THf | pad.
template <int D> struct McolRow {
    static constexpr int KK = (D + 3) / 4;
    static constexpr int RW = ((KK + 2 + 3) / 4) * 4; // floats per lane slot (16-byte units)
};

// BF (d <= 8): the Gram on ONE v_mfma_f32_16x16x32_bf16 per 16 x 16 block
// instead of KK = 2 f32 16x16x4 steps (16 instead of 64 cycles).  Each fp32
// coordinate is split x = hi + lo + r, hi = bf16(x), lo = bf16(x - hi)
// (x - hi exact in fp32), and the k = 32 slots hold all four products: A
// (columns) k-groups [hi | lo | hi | lo], B (rows) [hi | hi | lo | lo].
// |r| <= 2^-17 |x|: for x in [2^e, 2^(e+1)), |x - hi| <= 2^(e-8), so x - hi
// is either exactly 2^(e-8) (lo takes it, r = 0) or in a binade <= e - 9,
// where bf16's half-spacing is <= 2^(e-17).  Error of the fp32 value against
// h_j + xc_i.xc_j (S = sum_k |x_ik x_jk| <= nmax by Cauchy-Schwarz, |h_j| <=
// nmax / 2): h_j rounding 2^-25 nmax, fp32 inputs 2^-23 S, the split
// (|r_i||x_j| + |x_i||r_j| + |r_i r_j|) <= 2^-16 (1 + 2^-18) S, the bf16
// products exact in fp32 and at most 33 fp32 roundings of the sum over
// |h_j| + 1.02 S: in all <= 1.84e-5 nmax.  MCOL_DELTA_BF = 2^-15 nmax (1.66x
// that) plus 2^-100 for flushed denormals (tests/test_mcol_bf16_bound.py
// emulates the arithmetic; rounds 3-6 used 2^-14 from a 2^-16 |x| split
// bound).
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
// (the split itself: mcol_split_bf16, svgd_device.h; the centring writes
// every particle's two halves once per step, k_center_d's xs)

// The folded centre form (MIDC with a finite margin): the MFMA forms
// v = (h_j - TM) + sum_k (hi_i hi_j + lo_i hi_j + hi_i lo_j)_k + (p0 + p1 + p2)_i
// with p0 + p1 + p2 = fl32(-|xc_i|^2 / 2) split exactly into three bf16 parts
// (the fourth k-group of 8 slots, which the lo.lo products held: A [1 1 1 0 ..],
// B [p0 p1 p2 0 ..]) and TM, the bracket's centre, folded into the column
// operand C = fl32(h_j - TM) once per column block -- so v approximates
// x = e_ij - |xc_i|^2 / 2 - TM itself (e_ij = h_j + xc_i.xc_j, k_pair_rows'
// exact value), and one global half-width W classifies: no per-row
// thresholds, no subtraction per value.  Error of v against x (S = sum_k
// |x_ik x_jk| <= nmax): fp32 inputs 2^-23 S; the split without lo.lo:
// (hi + lo)_i (hi + lo)_j - x_i x_j is <= 2^-16 (1 + 2^-18) S and the
// dropped lo_i lo_j <= 2^-16 (1 + 2^-8)^2 S, together <= 1.01 * 2^-15 S;
// h_j, -|xc_i|^2/2 and h_j - TM rounded to fp32: 2^-25 nmax twice and 2^-24
// (nmax / 2 + |TM|); the products exact in fp32 and at most 28 nonzero terms
// summed (27 roundings) with partial sums below |h_j - TM| + 1.03 S + nmax / 2
// <= 2.03 nmax + |TM| <= 3.03 nmax (|TM| <= nmax, clamped): in all
// <= 3.62e-5 nmax.  MCOL_DELTA_FOLD = 2^-14 nmax (1.69x that) plus 2^-100;
// tests/test_mcol_bf16_bound.py emulates this arithmetic too.  With the fp64
// thresholds of k_pair_rows (e > TL_i = (n_i - lo + m_i) / 2 => key < lo;
// e <= TH_i = (n_i - hi - m_i) / 2 => key >= hi; m_i = 2^-48 (n_i + nmax) <=
// 2^-47 nmax), in x: below if x > -lo/2 - TM + m_i/2, above if x <= -hi/2
// - TM - m_i/2; so W = fp32_up(max(-lo/2 - TM, hi/2 + TM) + 2^-48 nmax +
// delta) gives v > W => below, v < -W => above, |v| <= W the band (a superset
// of the exact one: the fp64 finish decides it).  Padding rows carry p0 =
// -2^100 (never below or band); padding columns h = -inf (v = -inf).  A
// bracket without a lower or an upper end stages every pair (W = inf).
__device__ __forceinline__ uint4 mcol_fold_row(float q)
{
    uint32_t p[3];
    float r = q;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const __hip_bfloat162 h = __float22bfloat162_rn(make_float2(r, 0.0f));
        const uint32_t hb = *reinterpret_cast<const uint32_t *>(&h) & 0xffffu;
        p[k] = hb;
        r -= __uint_as_float(hb << 16);
    }
    return make_uint4(p[0] | (p[1] << 16), p[2], 0u, 0u);
}

// A block's 4 waves share one tile at a time: the tile's 256 rows live in LDS
// (B operands and thresholds, written when the row block changes), and wave w
// takes the 16-column blocks w, w + 4, ...  Each wave stages its own band
// pairs and owns region blockIdx * 4 + w, as k_pair_rows.
template <int D, bool BF = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BF ? 5 : D <= 8 ? 4 : 2, 8))) void k_pair_mcol(const double *__restrict__ xc,
                                                  const float *__restrict__ xf,
                                                  const uint4 *__restrict__ xs, int64_t n,
                                                  int64_t nb, int64_t t0, int64_t t1,
                                                  SinkCollect sc)
{
    constexpr int KP = med_rec_stride(D);  // fp64 records [xc | h | 0..]
    constexpr int KF = med_f32_stride(D);  // fp32 records [xc | h | 0..]
    constexpr int KK = McolRow<D>::KK;     // MFMA k-steps
    constexpr int RW = McolRow<D>::RW;
    constexpr int NI = PBLK / 16;          // 16-row blocks of a tile
    static_assert(!BF || (D <= 8 && RW == 4), "the bf16 split form takes d <= 8");
    __shared__ __attribute__((aligned(16))) float sRow[NI * 64 * RW]; // BF: the B fragments
    // BF: per row (TM, W) (the centre form, mcol_classify4m / _diag_m) or,
    // with delta = inf, (TLf, THf) -- 31 KiB of LDS in all: 5 work-groups
    // (waves) per CU
    constexpr bool MIDC = BF && SVGD_MCOL_CLS == 2;
    __shared__ float2 sT[BF ? PBLK : 1];
    __shared__ uint32_t sStage[4][MC_STG + 64]; // + the spill zone (SVGD_MCOL_STAGE)
    __shared__ uint32_t sBk[NBK];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int kq = lane >> 4, ql = lane & 15;
    uint32_t *stage = sStage[w];

    const uint64_t lo_key = sc.st->lo_key, hi_key = sc.st->hi_key;
    const double binv = sc.st->binv;
    const double nmax = __longlong_as_double((long long)*sc.nmax_bits);
    const double lo_d = __longlong_as_double((long long)lo_key);
    const double hi_d = hi_key >= 0x7ff0000000000000ull ? __builtin_inf()
                                                        : __longlong_as_double((long long)hi_key);
    const double delta = nmax > 0x1p40 ? __builtin_inf()
                         : BF     ? 0x1p-15 * nmax + 0x1p-100 // MCOL_DELTA_BF (above)
                                  : 4.0 * (D + 4) * 0x1p-24 * nmax + 0x1p-100;
    // the folded centre form (mcol_fold_row): TM and the one half-width W
    const bool fold = MIDC && delta < __builtin_inf();
    float TMf = 0.0f, Wf = __builtin_inff();
    if (fold && lo_key != 0 && hi_d < __builtin_inf()) {
        const double tm = fmin(fmax(-0.25 * (lo_d + hi_d), -nmax), nmax);
        TMf = (float)tm;
        const double dF = 0x1p-14 * nmax + 0x1p-100; // MCOL_DELTA_FOLD (above)
        Wf = f32_up(fmax(-0.5 * lo_d - (double)TMf, 0.5 * hi_d + (double)TMf) + 0x1p-48 * nmax + dF);
    }
    constexpr int AK = BF ? 4 : KK; // A operand dwords per lane (BF: 8 bf16)
    constexpr int BW = BF ? 2 : RW; // per-group row values kept in registers
    constexpr int TI = BF ? 0 : KK; // their (TLf, THf) slots
    if (sc.bpart)
        for (int e = tid; e < NBK; e += 256) sBk[e] = 0;

    const int64_t wreg = (int64_t)blockIdx.x * 4 + w;
    uint64_t *wregion = sc.region + wreg * sc.cap;
    int64_t wcnt = 0;             // keys written to the region
    unsigned long long below = 0; // below count (scalar: classified + exact)
    uint32_t vbelow = 0;          // SVGD_MCOL_CLS = 1: this lane's classified below values
    int scnt = 0;                 // staged band pairs
    bool ovf = false;             // a group outgrew the staging area

    // Staged entries: one per (lane, 16 x 16 block) holding band values --
    // row offset (bits 0..15) | column offset of the lane's 4 columns (16..27)
    // | which of the 4 are band pairs (28..31), all of the tile at rows ib,
    // columns jbase.  Each marked pair -> the exact fp64 key with
    // k_pair_rows' arithmetic (e = h_j + fma chain over k ascending,
    // s = max(fl(-2 h_i - 2 e), 0)), then below lo (counted) / in [lo, hi)
    // (appended to the region, bucketed) / dropped.
    auto flush = [&](int64_t ib, int64_t jbase) {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); // other lanes' staging stores
        if (scnt > MC_STG) { // entries went to the spill zone (SVGD_MCOL_STAGE >= 1)
            ovf = true;
            scnt = MC_STG;
        }
        for (int q0 = 0; q0 < (SVGD_MCOL_ABL == 3 ? 0 : scnt); q0 += 64) {
            const bool valid = q0 + lane < scnt;
            const uint32_t e = valid ? stage[q0 + lane] : 0u;
            uint32_t code = e >> 28; // 0 on invalid lanes
            const double *ri = xc + (valid ? ib + (e & 0xffffu) : 0) * KP;
            double xi[D + 1];
#pragma unroll
            for (int k = 0; k <= D; ++k) xi[k] = ri[k];
            const double ni = -2.0 * xi[D];
            const int64_t jl = jbase + ((e >> 16) & 0xfffu);
            // the lane's marked columns, lowest first (usually one)
            while (__any(code != 0)) {
                const bool act = code != 0;
                const int r = act ? __builtin_ctz(code) : 0;
                code &= code - 1u;
                const double *rj = xc + (act ? jl + r : 0) * KP;
                double ev = rj[D];
#pragma unroll
                for (int k = 0; k < D; ++k) ev = fma(xi[k], rj[k], ev);
                const uint64_t key = key_of(fmax(fma(-2.0, ev, ni), 0.0));
                below += __popcll(__ballot(act && key < lo_key));
                const bool keep = act && key >= lo_key && key < hi_key;
                const unsigned long long mk = __ballot(keep);
                if (keep) {
                    const int64_t pos = wcnt + __popcll(mk & ((1ull << lane) - 1ull));
                    if (pos < sc.cap) wregion[pos] = key;
                    if (sc.bpart) atomicAdd(&sBk[kbucket(key, lo_key, binv)], 1u);
                }
                wcnt += __popcll(mk);
            }
        }
        scnt = 0;
        __builtin_amdgcn_s_waitcnt(0xF70); // vmcnt(0): the flush's stores drained here, once (see the column loop)
    };

    // lane-constant part of "j > i" inside a 16 x 16 block (diagonal tiles):
    // j - i = (4 kq - ql) + r + (jl0 - il0)
    const int xl = 4 * kq - ql;
    // Schedule (L2 locality, as k_pair_tcol; the plan's tile SET [t0, t1) is
    // unchanged): the rank's tile rows I (plan.cpp: row I holds slots
    // 0..cnt(I)-1, J = I + slot mod nb) are cut into bands of R rows dealt
    // round-robin to the nG = 8 XCDs (block b runs on XCD b % 8).  Inside a
    // band the XCD's P blocks sweep the slots together: block q keeps row
    // I = band + q % R (its rows stay in LDS for the whole band) and takes
    // slots q / R, q / R + S, ... (S = P / R), so at any moment the XCD's
    // blocks read ~R + S neighbouring column tiles, each shared by ~R blocks
    // through the XCD's L2 -- instead of P unrelated column streams (each XCD
    // re-fetched the fp32 records ~17 times per pass: 430 MB at cfg3).
    const int G = gridDim.x;
    const int nG = (G % 8 == 0) ? 8 : 1;
    const int P = G / nG, gx = blockIdx.x % nG, q = blockIdx.x / nG;
    const int64_t H = (nb - 1) / 2;
    const int64_t half = (nb & 1) == 0 ? nb / 2 : 0, c1 = H + 2, c2 = H + 1;
    int64_t Ia = 0, Ib = -1;
    if (t1 > t0) {
        int64_t Jd;
        tile_coords(nb, t0, &Ia, &Jd);
        tile_coords(nb, t1 - 1, &Ib, &Jd);
    }
    int R = 32;
    while (P % R) R >>= 1;
    while (R > 1 && Ib - Ia + 1 < (int64_t)nG * R) R >>= 1; // every XCD gets a band
    const int S = P / R, rr = q % R, ph = q / R;
    const int64_t nbands = (Ib - Ia + 1 + R - 1) / R;
    struct Pos {
        int64_t k, I, s, J, hi;
    };
    // the first tile at or after band p.k of this block's row and phase
    auto enter_row = [&](Pos &p) {
        for (; p.k < nbands; p.k += nG) {
            const int64_t I = Ia + p.k * R + rr;
            if (I > Ib) continue;
            const int64_t rs = I < half ? I * c1 : half * c1 + (I - half) * c2;
            const int64_t lo = max<int64_t>(0, t0 - rs);
            const int64_t hi = min<int64_t>(I < half ? c1 : c2, t1 - rs);
            const int64_t sl = lo <= ph ? ph : ph + (lo - ph + S - 1) / S * S;
            if (sl < hi) {
                p.I = I;
                p.s = sl;
                p.hi = hi;
                p.J = I + sl >= nb ? I + sl - nb : I + sl;
                return true;
            }
        }
        return false;
    };
    auto advance = [&](Pos &p) {
        p.s += S;
        if (p.s < p.hi) {
            p.J = p.I + p.s >= nb ? p.I + p.s - nb : p.I + p.s;
            return true;
        }
        p.k += nG;
        return enter_row(p);
    };
    Pos pos{gx, 0, 0, 0, 0};
    if (t1 > t0 && enter_row(pos)) {
        int64_t curI = -1;
        do {
            const int64_t I = pos.I, J = pos.J;
            const int64_t ib = I * PBLK, jbase = J * PBLK;
            if (I != curI) {
                // the tile's rows: lane slot (b, l) of row ib + 16 b + (l & 15)
                __syncthreads(); // every wave is done with the previous rows
                for (int e = tid; e < NI * 64; e += 256) {
                    const int b = e >> 6, l = e & 63;
                    const int64_t i = ib + 16 * b + (l & 15);
                    const bool iv = i < n;
                    const int64_t ic = iv ? i : n - 1;
                    float *o = sRow + e * RW;
                    if constexpr (BF) {
                        // B fragment: k-groups [hi | hi | lo | lo] of row i, or
                        // [hi | hi | lo | -|x_i|^2/2 in 3 parts] (fold)
                        if (fold && (l >> 4) == 3)
                            *reinterpret_cast<uint4 *>(o) =
                                mcol_fold_row(iv ? (float)xc[ic * KP + D] : -0x1p100f);
                        else
                            *reinterpret_cast<uint4 *>(o) = xs[2 * ic + ((l >> 4) >= 2 ? 1 : 0)];
                        if (!fold && e < PBLK) { // thresholds once per row: row ib + e
                            const int64_t it = ib + e;
                            const bool tv = it < n;
                            const int64_t tc = tv ? it : n - 1;
                            const double ni = -2.0 * xc[tc * KP + D];
                            const double m = 0x1p-48 * (ni + nmax);
                            const double TL = lo_key == 0 ? __builtin_inf() : 0.5 * (ni - lo_d + m);
                            const double TH = 0.5 * (ni - hi_d - m);
                            const float2 t = make_float2(tv ? f32_up(TL + delta) : __builtin_inff(),
                                                         tv ? f32_down(TH - delta) : __builtin_inff());
                            sT[e] = t;
                        }
                        continue;
                    }
#pragma unroll
                    for (int kk = 0; kk < KK; ++kk) {
                        const int k = 4 * kk + (l >> 4);
                        o[kk] = k < D ? xf[ic * KF + k] : 0.0f; // slot D holds h
                    }
                    const double ni = -2.0 * xc[ic * KP + D];
                    const double m = 0x1p-48 * (ni + nmax);
                    const double TL = lo_key == 0 ? __builtin_inf() : 0.5 * (ni - lo_d + m);
                    const double TH = 0.5 * (ni - hi_d - m);
                    o[KK] = iv ? f32_up(TL + delta) : __builtin_inff();
                    o[KK + 1] = iv ? f32_down(TH - delta) : __builtin_inff();
                }
                __syncthreads();
                curI = I;
            }
            const bool diag = I == J;
            const int njb = (int)min<int64_t>(PBLK / 16, (n - jbase + 15) / 16);
            // this wave's 16-column blocks; the next one's operands load during
            // the current one's MFMAs (xf rows [n, np) hold h = -inf: padding
            // columns are never below or in the band; blocks end before np)
            auto load_cols = [&](int jb, float (&A)[AK], f4 &hq) {
                const float *xcol = xf + (jbase + 16 * jb) * KF;
                if constexpr (BF) {
                    // A fragment: k-groups [hi | lo | hi | lo] of column j (the
                    // centring's split: one 16-byte load instead of 64 bytes
                    // and ~45 VALU per column block)
                    *reinterpret_cast<uint4 *>(A) =
                        fold && kq == 3 ? make_uint4(0x3f803f80u, 0x3f80u, 0u, 0u) // [1 1 1 0 ..]
                                        : xs[2 * (jbase + 16 * jb + ql) + (kq & 1)];
#pragma unroll
                    for (int r = 0; r < 4; ++r) hq[r] = xcol[(4 * kq + r) * KF + D] - TMf; // (TMf = 0 unfolded)
                    return;
                }
#pragma unroll
                for (int kk = 0; kk < KK; ++kk) {
                    const float x = xcol[ql * KF + 4 * kk + kq];
                    A[kk] = (4 * kk + kq == D) ? 0.0f : x; // slot D holds h
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) hq[r] = xcol[(4 * kq + r) * KF + D];
            };
            // one group of MC_NG row blocks: its row operands from LDS, its MFMAs
            // (BF: the row values sT hold the form the launch classifies with)
            auto group_mfma = [&](auto mid_tag, int g0, const f4 &hq, const float (&A)[AK],
                                  float (&Bg)[MC_NG][BW], f4 (&acc)[MC_NG]) {
                if constexpr (BF) {
                    constexpr bool MID = decltype(mid_tag)::value;
                    const bf16x8_t a = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4 *>(A));
#pragma unroll
                    for (int g = 0; g < MC_NG; ++g) {
                        const uint4 b = *reinterpret_cast<const uint4 *>(sRow + ((g0 + g) * 64 + lane) * RW);
                        if constexpr (!MID) { // (the folded form has no per-row values)
                            const float2 t = sT[16 * (g0 + g) + ql];
                            Bg[g][0] = t.x;
                            Bg[g][1] = t.y;
                        }
                        acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8_t, b), hq,
                                                                         0, 0, 0);
                    }
                    return;
                }
#pragma unroll
                for (int g = 0; g < MC_NG; ++g)
#pragma unroll
                    for (int q = 0; q < RW; q += 4)
                        *reinterpret_cast<f4 *>(&Bg[g][q]) =
                            *reinterpret_cast<const f4 *>(sRow + ((g0 + g) * 64 + lane) * RW + q);
                // k-step outer, row block inner: the MC_NG chains interleave,
                // so no MFMA waits for the one before it (dependent-accumulator
                // latency 40 cycles); each chain still runs k ascending
#pragma unroll
                for (int g = 0; g < MC_NG; ++g) acc[g] = hq;
#pragma unroll
                for (int kk = 0; kk < KK; ++kk)
#pragma unroll
                    for (int g = 0; g < MC_NG; ++g)
                        acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[kk], Bg[g][kk], acc[g], 0, 0, 0);
            };
            // Per 16-column block: the groups' MFMAs run one group ahead of the
            // classification (phase 2: two compares per value straight into
            // lane masks -- below (v > TLf) counted on the scalar unit, band (v
            // > THf but not below) OR-ed; phase 3, rare: stage the band pairs).
            auto jloop = [&](auto diag_tag, auto mid_tag) {
                constexpr bool DIAG = decltype(diag_tag)::value;
                constexpr bool MID = decltype(mid_tag)::value;
                float A[AK], An[AK];
                f4 hq, hqn;
                if (w < njb) load_cols(w, A, hq);
                // vmcnt(0): the column loop starts with no memory operation in
                // flight (the compiler's wait placement is path-insensitive at
                // the loop head: with these first operands, or the flush's
                // stores, possibly pending it waited for EVERYTHING -- the
                // next column block's prefetch included -- at the top of every
                // iteration)
                __builtin_amdgcn_s_waitcnt(0xF70);
                for (int jb = w; jb < njb; jb += 4) {
                    // (a block of 16 x 256 pairs stages ~10 band pairs; one that
                    // outgrows the area marks the region overflowed)
                    if (scnt > MC_STG / 2) flush(ib, jbase);
                    if (jb + 4 < njb) load_cols(jb + 4, An, hqn);
                    const int jl0 = 16 * jb;
                    // the lane's part of a staged entry for this column block
                    // (row offset | the lane's 4-column offset << 16)
                    const uint32_t ebase = (uint32_t)ql | ((uint32_t)(jl0 + 4 * kq) << 16);
                    float Bg[MC_NG][BW], Bn[MC_NG][BW];
                    f4 acc[MC_NG], accn[MC_NG];
                    group_mfma(mid_tag, 0, hq, A, Bg, acc);
                    // unrolled: the next group's accumulators and row values
                    // take other registers instead of being copied each group
#pragma unroll
                    for (int g0 = 0; g0 < NI; g0 += MC_NG) {
                        if (g0 + MC_NG < NI) group_mfma(mid_tag, g0 + MC_NG, hq, A, Bn, accn);
                        uint32_t nbelow = 0;
#pragma unroll
                        for (int g = 0; g < MC_NG; ++g) {
                            unsigned long long h[4], any = 0, lb[4]; // (lb: the below masks, unused)
                            float xm[4]; // MID: v - TM
                            if constexpr (SVGD_MCOL_ABL == 2) {
                                asm volatile("" ::"v"(acc[g][0]), "v"(acc[g][1]), "v"(acc[g][2]),
                                             "v"(acc[g][3]), "v"(Bg[g][TI]), "v"(Bg[g][TI + 1]));
                                continue;
                            } else if constexpr (DIAG && MID) {
#pragma unroll
                                for (int r = 0; r < 4; ++r) {
                                    h[r] = mcol_classify_diag_m(acc[g][r], Wf, xl, 16 * (g0 + g) - jl0 - r, nbelow);
                                    any |= h[r];
                                }
                            } else if constexpr (DIAG) {
#pragma unroll
                                for (int r = 0; r < 4; ++r) {
                                    h[r] = mcol_classify_diag(acc[g][r], Bg[g][TI], Bg[g][TI + 1], xl,
                                                              16 * (g0 + g) - jl0 - r, nbelow);
                                    any |= h[r];
                                }
                            } else if constexpr (MID) {
#pragma unroll
                                for (int r = 0; r < 4; ++r) xm[r] = acc[g][r]; // (folded: v is x)
                                any = mcol_classify4m(xm, Wf, nbelow, lb);
                            } else if constexpr (SVGD_MCOL_CLS == 1) {
                                uint32_t bv[4];
                                mcol_classify4v(acc[g], Bg[g][TI], Bg[g][TI + 1], vbelow, bv);
                                any = __ballot((int)(bv[0] | bv[1] | bv[2] | bv[3]) < 0);
                                if (__builtin_expect(any != 0, 0)) {
                                    // the lane masks the staging takes (rare)
#pragma unroll
                                    for (int r = 0; r < 4; ++r) h[r] = __ballot((int)bv[r] < 0);
                                }
                            } else {
                                any = mcol_classify4(acc[g], Bg[g][TI], Bg[g][TI + 1], nbelow, h);
                            }
                            // ~0.4 of the blocks hold band values (~1 pair each):
                            // ONE entry per lane with its 4 values' band bits (the
                            // flush expands the bits)
                            if constexpr (SVGD_MCOL_STAGE >= 1 && (SVGD_MCOL_ABL == 0 || SVGD_MCOL_ABL == 3)) {
                                if (SVGD_MCOL_STAGE == 2 || __builtin_expect(any != 0, 0)) {
                                    // every lane stores: a lane without band values, or an
                                    // entry past the area, lands in the spill zone; the
                                    // flush reports an overflowed area (scnt > MC_STG)
                                    if constexpr (MID && !DIAG) mcol_band4m(xm, Wf, h);
                                    const uint32_t code = mcol_code4(h);
                                    const uint32_t pre = __builtin_amdgcn_mbcnt_hi(
                                        (uint32_t)(any >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)any, 0u));
                                    // a lane holding band values (its bit in any) takes the next
                                    // slot, the others the spill zone
                                    const uint32_t idx = min(mcol_sel(any, (uint32_t)scnt + pre, (uint32_t)(MC_STG + lane)),
                                                             (uint32_t)(MC_STG + lane));
                                    stage[idx] = (ebase + 16u * (g0 + g)) | (code << 28);
                                    scnt += __popcll(any);
                                }
                            } else if ((SVGD_MCOL_ABL == 0 || SVGD_MCOL_ABL == 3) && __builtin_expect(any != 0, 0)) {
                                // ~0.4 of the blocks, ~1 band pair each: ONE entry per
                                // lane holding band values (its 4 values' band bits)
                                const int c = __popcll(any);
                                if (scnt + c > MC_STG) { // pathological band: give up
                                    ovf = true;          // (region overflow -> exact fallback)
                                } else {
                                    if constexpr (MID && !DIAG) mcol_band4m(xm, Wf, h);
                                    const uint32_t code = mcol_code4(h);
                                    const uint32_t pre = __builtin_amdgcn_mbcnt_hi(
                                        (uint32_t)(any >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)any, 0u));
                                    if (code)
                                        stage[scnt + pre] = (16u * (g0 + g) + ql) |
                                                            ((uint32_t)(jl0 + 4 * kq) << 16) | (code << 28);
                                    scnt += c;
                                }
                            }
                        }
                        below += nbelow;
#pragma unroll
                        for (int g = 0; g < MC_NG; ++g) {
                            acc[g] = accn[g];
#pragma unroll
                            for (int q = 0; q < BW; ++q) Bg[g][q] = Bn[g][q];
                        }
                    }
#pragma unroll
                    for (int kk = 0; kk < AK; ++kk) A[kk] = An[kk];
                    hq = hqn;
                }
            };
            if constexpr (MIDC) {
                // delta = inf (nmax > 2^40): values may exceed mcol_classify4m's
                // range -- the lane-mask form (sT holds (TLf, THf) then)
                if (delta < __builtin_inf()) {
                    if (diag)
                        jloop(std::true_type{}, std::true_type{});
                    else
                        jloop(std::false_type{}, std::true_type{});
                } else if (diag) {
                    jloop(std::true_type{}, std::false_type{});
                } else {
                    jloop(std::false_type{}, std::false_type{});
                }
            } else if (diag) {
                jloop(std::true_type{}, std::false_type{});
            } else {
                jloop(std::false_type{}, std::false_type{});
            }
            if (scnt) flush(ib, jbase);
        } while (advance(pos));
    }

    if (SVGD_MCOL_CLS == 1) { // the lanes' classified below counts
        unsigned long long vb = vbelow;
        for (int o = 32; o > 0; o >>= 1) vb += __shfl_xor(vb, o);
        below += vb;
    }
    if (lane == 0) {
        sc.below_out[wreg] = below;
        // an overflowed staging area reports an overflowed region: the host
        // then takes the exact streamed fallback
        sc.count_out[wreg] = ovf ? 0xffffffffu : (uint32_t)min<int64_t>(wcnt, 0xffffffffll);
    }
    if (sc.bpart) {
        __syncthreads();
        for (int e = tid; e < NBK; e += 256) sc.bpart[(int64_t)blockIdx.x * NBK + e] = sBk[e];
    }
}


// ============================== fp32 tile-path collect (d > 16, SVGD_F32) ==
//
// The bracket collect pass (MODE 0 of k_pair_tiles<float>) with the same
// arithmetic, so every pass (sample tiles, radix fallback, this) forms the
// same fp32 key: dot = the MFMA chain over k ascending from 0 (A = 16
// columns j, B = 16 rows i, lane l: x[.. + l%16][4kk + l/16]), then
// s = max(fma(-2, dot, n_i + n_j), 0) (GaussianRBFKernel.hpp:179-187).  Here
// the sign is flipped, v = min(fma(2, dot, (-n_i) + (-n_j)), 0) = -s exactly
// (negation commutes with round-to-nearest), so the lane-mask classifier of
// k_pair_mcol applies unchanged: below <=> s < loT <=> v > -loT, candidate <=>
// v > -hiT; the key of a candidate is key_of(|v|) = key_of(s).
//
// A wave owns one 16-column block of every tile of its block and keeps the
// tile's 64 rows (4 row blocks of B operands, KP floats each) in VGPRs across
// the run of tiles that share them (~nb/2); the next tile's columns load
// during the current one's 4 x KP/4 MFMAs.  No LDS traffic, no barriers in
// the loop: the pass is MFMA-issue bound (16 x 16 x KP pairs per 4KP MFMA
// cycles).  Candidates (the band, ~0.3 %) go straight to the block's region.
// Rows / columns >= n carry norm -inf: never below, never candidates.
constexpr int TC_STG = 512; // staged band values per wave (k_pair_tcol)

template <int KP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_pair_tcol(
    const float *__restrict__ xc, const float *__restrict__ nrm, int64_t n, int64_t nb, int64_t t0,
    int64_t t1, SinkCollect sc)
{
    constexpr int KK = KP / 4;
    __shared__ uint32_t sBk[NBK];
    __shared__ uint32_t sCnt;
    __shared__ unsigned long long sBelow[4];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int kq = lane >> 4, ql = lane & 15;

    const uint64_t lo_key = sc.st->lo_key, hi_key = sc.st->hi_key;
    const double binv = sc.st->binv;
    const double lo_d = __longlong_as_double((long long)lo_key);
    const double hi_d = hi_key >= 0x7ff0000000000000ull ? __builtin_inf()
                                                        : __longlong_as_double((long long)hi_key);
    // the smallest floats >= the bracket's doubles (as k_pair_tiles), negated
    float loT = (float)lo_d, hiT = (float)hi_d;
    if ((double)loT < lo_d) loT = __int_as_float(__float_as_int(loT) + 1);
    if ((double)hiT < hi_d) hiT = __int_as_float(__float_as_int(hiT) + 1);
    // v = fma(2, dot, -n_i - n_j) = -(the unclamped s): min(v, 0) > -T <=>
    // v > -T for T > 0, and never for T = 0 (+inf then), so the clamp is left
    // to the key of the staged band values
    const float tl = loT > 0.0f ? -loT : __builtin_inff();
    const float th = hiT > 0.0f ? -hiT : __builtin_inff();
    __shared__ float sStage[4][TC_STG];
    float *stage = sStage[w];
    int scnt = 0; // staged band values of this wave
    if (tid == 0) sCnt = 0;
    if (sc.bpart)
        for (int e = tid; e < NBK; e += 256) sBk[e] = 0;
    __syncthreads();

    uint64_t *region = sc.region + (int64_t)blockIdx.x * sc.cap;
    // scalar, 64-bit: one wave may classify more than 2^32 pairs (a small
    // collect grid, or large N at d > 16)
    unsigned long long below = 0;
    const int xl = 4 * kq - ql; // j - i = xl + r + 16 (w - rb) on diagonal tiles
    const float ninf = -__builtin_inff();

    // A column block: the MFMA A operands and the raw norms, loaded
    // unconditionally (rows < np) and masked at use -- a select right after
    // the load would make the compiler wait for it (and the whole prefetch)
    struct Cols {
        float A[KK];
        f4 nv;
    };
    auto load_cols = [&](int J, Cols &c) {
        const int64_t j0 = (int64_t)J * TB + 16 * w;
        if constexpr (KP % 16 == 0) { // kslot order: 16-byte loads
            const float *xcol = xc + (j0 + ql) * KP + 4 * kq;
#pragma unroll
            for (int u = 0; u < KK / 4; ++u) {
                const f4 t = *reinterpret_cast<const f4 *>(xcol + 16 * u);
#pragma unroll
                for (int e = 0; e < 4; ++e) c.A[4 * u + e] = t[e];
            }
        } else {
            const float *xcol = xc + (j0 + ql) * KP;
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) c.A[kk] = xcol[kslot<float, KP>(kk, kq)];
        }
        c.nv = *reinterpret_cast<const f4 *>(nrm + j0 + 4 * kq);
    };

    // Schedule (L2 locality; the plan's tile SET [t0, t1) is unchanged): the
    // rank's tile rows I (plan.cpp: row I holds slots 0..cnt(I)-1, J = I +
    // slot mod nb) are cut into bands of R rows, dealt round-robin to the
    // nG = 8 XCDs (block b runs on XCD b % 8).  Inside a band the XCD's P
    // blocks sweep the slots together: block q keeps row I = band + q % R
    // (its rows stay in VGPRs for the whole band) and takes slots q / R,
    // q / R + S, ... (S = P / R).  At any moment the XCD's blocks read ~R + S
    // neighbouring column blocks, each shared by ~R blocks through its L2,
    // instead of P unrelated column streams (15 % L2 hits measured).
    const int G = gridDim.x;
    const int nG = (G % 8 == 0) ? 8 : 1;
    const int P = G / nG, g = blockIdx.x % nG, q = blockIdx.x / nG;
    int R = 32;
    while (P % R) R >>= 1;
    const int S = P / R, rr = q % R, ph = q / R;
    const int nb32 = (int)nb, n32 = (int)min<int64_t>(n, 0x7fffffff);
    const int64_t H = (nb - 1) / 2;
    const int64_t half = (nb & 1) == 0 ? nb / 2 : 0, c1 = H + 2, c2 = H + 1;
    int Ia = 0, Ib = -1;
    if (t1 > t0) {
        int64_t I64, Jd;
        tile_coords(nb, t0, &I64, &Jd);
        Ia = (int)I64;
        tile_coords(nb, t1 - 1, &I64, &Jd);
        Ib = (int)I64;
    }
    const int nbands = (Ib - Ia + 1 + R - 1) / R;
    // scalar position in the schedule; slots s < hi of row I, column block J
    struct Pos {
        int k, I, s, J, hi;
    };
    // the first tile at or after band p.k (64-bit plan arithmetic once per row)
    auto enter_row = [&](Pos &p) {
        for (; p.k < nbands; p.k += nG) {
            const int I = Ia + p.k * R + rr;
            if (I > Ib) continue;
            const int64_t rs = I < half ? I * c1 : half * c1 + (I - half) * c2;
            const int lo = (int)max<int64_t>(0, t0 - rs);
            const int hi = (int)min<int64_t>(I < half ? c1 : c2, t1 - rs);
            const int s = lo <= ph ? ph : ph + (lo - ph + S - 1) / S * S;
            if (s < hi) {
                p.I = I;
                p.s = s;
                p.hi = hi;
                p.J = I + s >= nb32 ? I + s - nb32 : I + s;
                return true;
            }
        }
        return false;
    };
    auto advance = [&](Pos &p) {
        p.s += S;
        if (p.s < p.hi) {
            p.J = p.I + p.s >= nb32 ? p.I + p.s - nb32 : p.I + p.s;
            return true;
        }
        p.k += nG;
        return enter_row(p);
    };

    // staged band values -> keys (s = max(-v, 0), as k_pair_tiles' fmax) in
    // the block's region (one LDS atomic per 64) and the bucket histogram
    auto flush = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); // other lanes' staging stores
        for (int q0 = 0; q0 < scnt; q0 += 64) {
            const int c = min(64, scnt - q0);
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(&sCnt, (uint32_t)c);
            base = __shfl(base, 0);
            if (lane < c) {
                const float v = stage[q0 + lane];
                const uint64_t key = key_of((double)(v >= 0.0f ? 0.0f : -v));
                const int64_t pos = (int64_t)base + lane;
                if (pos < sc.cap) region[pos] = key;
                if (sc.bpart) atomicAdd(&sBk[kbucket(key, lo_key, binv)], 1u);
            }
        }
        scnt = 0;
        __builtin_amdgcn_s_waitcnt(0xF70); // vmcnt(0): the flush's stores drained here, once (see the column loop)
    };

    // the tile row's B operands, shared by the block's 4 waves (written at a
    // row change, between barriers: every wave follows the same schedule)
    __shared__ float sB[4 * KK * 64];
    float hr[4];
    // one tile (I, J): 4 x KK MFMAs, then the classification
    auto tile = [&](const Pos &p, const Cols &c) {
        const int j0 = p.J * TB + 16 * w + 4 * kq;
        float hc[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) hc[r] = j0 + r < n32 ? -c.nv[r] : ninf;
        f4 acc[4];
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) acc[rb] = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
#pragma unroll
            for (int rb = 0; rb < 4; ++rb)
                acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(c.A[kk], sB[(rb * KK + kk) * 64 + lane],
                                                               acc[rb], 0, 0, 0);
        const bool diag = p.s == 0;
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
            // packed fp32 (v_pk_add_f32 / v_pk_fma_f32): the same roundings,
            // half the instructions
            typedef float f2 __attribute__((ext_vector_type(2)));
            const f2 hh = {hr[rb], hr[rb]}, two = {2.0f, 2.0f};
            const f2 t01 = hh + f2{hc[0], hc[1]}, t23 = hh + f2{hc[2], hc[3]};
            const f2 v01 = __builtin_elementwise_fma(two, f2{acc[rb][0], acc[rb][1]}, t01);
            const f2 v23 = __builtin_elementwise_fma(two, f2{acc[rb][2], acc[rb][3]}, t23);
            const f4 v = {v01[0], v01[1], v23[0], v23[1]};
            // lane masks: below counted on the scalar unit, band lanes OR-ed
            // (measured faster than per-lane vector counters: 2.7 vs 3.2 ms)
            unsigned long long h[4], any = 0;
            uint32_t nbl = 0;
            if (diag) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    h[r] = mcol_classify_diag(v[r], tl, th, xl, 16 * rb - 16 * w - r, nbl);
                    any |= h[r];
                }
            } else {
                any = mcol_classify4(v, tl, th, nbl, h);
            }
            below += nbl;
            // band values (~1 % of the pairs) are staged; their keys are
            // formed and written in batches of 64 (flush).  A row block adds
            // at most 256 (a bracket holding every pair: the direct path)
            if (__builtin_expect(any != 0, 0)) {
                if (scnt > TC_STG - 256) flush();
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const unsigned long long m = h[r];
                    if (!m) continue;
                    if ((m >> lane) & 1ull) stage[scnt + __popcll(m & ((1ull << lane) - 1ull))] = v[r];
                    scnt += __popcll(m);
                }
            }
        }
    };
    auto rows = [&](int I) {
        const int ib = I * TB;
        __syncthreads(); // every wave is done with the previous row
        for (int e = tid; e < 4 * KK * 64; e += 256) {
            const int l = e & 63, kk = (e >> 6) % KK, rb = (e >> 6) / KK;
            sB[e] = xc[(int64_t)(ib + 16 * rb + (l & 15)) * KP + kslot<float, KP>(kk, l >> 4)];
        }
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
            const int i = ib + 16 * rb + ql;
            const float nv = nrm[i];
            hr[rb] = i < n32 ? -nv : ninf;
        }
        __syncthreads();
        // all loads done (vmcnt(0) expcnt(7) lgkmcnt(15)): the waits inside
        // the slot loop then only ever cover the current column buffer
        __builtin_amdgcn_s_waitcnt(0x0F70);
    };

    // Per row: its B operands, then its slots two at a time over two column
    // buffers (no register copies in the loop): the next tile's columns load
    // during the current tile's MFMAs.  The prefetch is issued on every path
    // (block 0 when there is no next tile) so the compiler's wait for the
    // current buffer never includes it.
    Pos p0{g, 0, 0, 0, 0};
    if (enter_row(p0)) {
        Cols c0, c1;
        load_cols(p0.J, c0);
        for (bool live = true; live;) {
            rows(p0.I);
            for (;;) {
                Pos p1 = p0;
                const bool m1 = advance(p1);
                load_cols(m1 ? p1.J : 0, c1);
                __builtin_amdgcn_sched_barrier(0); // the prefetch issues before the MFMAs
                tile(p0, c0);
                if (!m1) {
                    live = false;
                    break;
                }
                if (p1.I != p0.I) { // next row: its first columns are in c1
                    p0 = p1;
                    c0 = c1;
                    break;
                }
                Pos p2 = p1;
                const bool m2 = advance(p2);
                load_cols(m2 ? p2.J : 0, c0);
                __builtin_amdgcn_sched_barrier(0);
                tile(p1, c1);
                if (!m2) {
                    live = false;
                    break;
                }
                const bool row_end = p2.I != p1.I;
                p0 = p2;
                if (row_end) break;
            }
        }
    }

    if (scnt) flush();
    if (lane == 0) sBelow[w] = below;
    __syncthreads();
    if (tid == 0) {
        sc.below_out[blockIdx.x] = sBelow[0] + sBelow[1] + sBelow[2] + sBelow[3];
        sc.count_out[blockIdx.x] = sCnt;
    }
    if (sc.bpart)
        for (int e = tid; e < NBK; e += 256) sc.bpart[(int64_t)blockIdx.x * NBK + e] = sBk[e];
}


// ======================= F32 bf16-key collect (KP 32 / 64: d > 16, SVGD_F32) ==
//
// The bracket collect pass over the bf16 part-product keys (svgd_device.h
// "F32 pair keys"; the keys k_pair_tiles<float> forms at these KP): per
// 64 x 16 wave tile 4 x 6 KP/32 v_mfma_f32_16x16x32_bf16 of 16 cycles (the
// fp32 form: 4 x KP/4 f32 MFMAs of 32).  The wave's 16 columns' parts in
// VGPRs (from xk, the next tile's loading during the current one's MFMAs),
// the tile row's 4 row blocks' parts in VGPRs too, for the whole run of
// tiles sharing the row (no LDS reads per tile); a wrapped tile (J < I) gives the rows (the larger
// indices) the A role, which transposes the lane map: row 4 kq + r, column ql.
// Each tile kind (plain, wrapped, diagonal) is its own straight-line code.
// Norms come from nrmf, whose padding rows hold +inf (launch_cvt_nrm_f32):
// a padding row or column gives v = -inf, never below, never in the band.
// Band values are staged one 16-byte entry per lane and row block (its 4
// values, NaN where not a band value: a band value is never NaN), so a row
// block with band values costs one masked-free store; the flush keys them.
constexpr int TC3_ENT = 448; // staged entries per wave (+ 64 spill slots); a tile adds <= 256

// XCD-banded tile schedule of the tile-path collects (k_pair_tcol's, as a
// struct): the rank's tile rows I (plan.cpp: row I holds slots
// 0..cnt(I)-1, J = I + slot mod nb) in bands of R rows dealt round-robin to
// the 8 XCDs; inside a band the XCD's P blocks sweep the slots together
// (block q keeps row I = band + q % R and takes slots q / R, q / R + S, ...).
struct TileSched {
    int nG, R, S, rr, ph, nb32, Ia, Ib, nbands;
    int64_t t0, t1, half, c1, c2;
    struct Pos {
        int k, I, s, J, hi;
    };
    __device__ TileSched(int64_t nb, int64_t t0_, int64_t t1_) : t0(t0_), t1(t1_)
    {
        const int G = gridDim.x;
        nG = (G % 8 == 0) ? 8 : 1;
        const int P = G / nG, q = blockIdx.x / nG;
        R = 32;
        while (P % R) R >>= 1;
        S = P / R;
        rr = q % R;
        ph = q / R;
        nb32 = (int)nb;
        const int64_t H = (nb - 1) / 2;
        half = (nb & 1) == 0 ? nb / 2 : 0;
        c1 = H + 2;
        c2 = H + 1;
        Ia = 0;
        Ib = -1;
        if (t1 > t0) {
            int64_t I64, Jd;
            tile_coords(nb, t0, &I64, &Jd);
            Ia = (int)I64;
            tile_coords(nb, t1 - 1, &I64, &Jd);
            Ib = (int)I64;
        }
        nbands = (Ib - Ia + 1 + R - 1) / R;
    }
    __device__ Pos first() const { return Pos{(int)(blockIdx.x % nG), 0, 0, 0, 0}; }
    // the first tile at or after band p.k (64-bit plan arithmetic once per row)
    __device__ bool enter_row(Pos &p) const
    {
        for (; p.k < nbands; p.k += nG) {
            const int I = Ia + p.k * R + rr;
            if (I > Ib) continue;
            const int64_t rs = I < half ? I * c1 : half * c1 + (I - half) * c2;
            const int lo = (int)max<int64_t>(0, t0 - rs);
            const int hi = (int)min<int64_t>(I < half ? c1 : c2, t1 - rs);
            const int s = lo <= ph ? ph : ph + (lo - ph + S - 1) / S * S;
            if (s < hi) {
                p.I = I;
                p.s = s;
                p.hi = hi;
                p.J = I + s >= nb32 ? I + s - nb32 : I + s;
                return true;
            }
        }
        return false;
    }
    __device__ bool advance(Pos &p) const
    {
        p.s += S;
        if (p.s < p.hi) {
            p.J = p.I + p.s >= nb32 ? p.I + p.s - nb32 : p.I + p.s;
            return true;
        }
        p.k += nG;
        return enter_row(p);
    }
};

// 1 in the lanes whose bit is set in the wave mask m (one v_cndmask)
__device__ __forceinline__ uint32_t lane_bit(unsigned long long m)
{
    uint32_t b;
    asm volatile("v_cndmask_b32_e64 %0, 0, 1, %1" : "=v"(b) : "s"(m));
    return b;
}
// v where the mask bit is set, else x (one v_cndmask)
__device__ __forceinline__ float lane_sel(unsigned long long m, float v, float x)
{
    float r;
    asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(v), "s"(m));
    return r;
}

template <int KP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 8))) void k_pair_tcol3(
    const float *__restrict__ nrm, const uint32_t *__restrict__ xk, int64_t n, int64_t nb, int64_t t0,
    int64_t t1, SinkCollect sc)
{
    constexpr int NDB = KP / 32;
    static_assert(kb3_keys(KP), "the bf16-key collect takes KP 32 / 64");
    __shared__ uint32_t sBk[NBK];
    __shared__ uint32_t sCnt;
    __shared__ unsigned long long sBelow[4];
    __shared__ f4 sStage[4][TC3_ENT + 64];                   // + the spill zone
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int kq = lane >> 4, ql = lane & 15;

    const uint64_t lo_key = sc.st->lo_key, hi_key = sc.st->hi_key;
    const double binv = sc.st->binv;
    const double lo_d = __longlong_as_double((long long)lo_key);
    const double hi_d = hi_key >= 0x7ff0000000000000ull ? __builtin_inf()
                                                        : __longlong_as_double((long long)hi_key);
    // the smallest floats >= the bracket's doubles (as k_pair_tiles), negated
    // (k_pair_tcol's classification: v = fma(2, dot, -n_i - n_j) = -s)
    float loT = (float)lo_d, hiT = (float)hi_d;
    if ((double)loT < lo_d) loT = __int_as_float(__float_as_int(loT) + 1);
    if ((double)hiT < hi_d) hiT = __int_as_float(__float_as_int(hiT) + 1);
    const float tl = loT > 0.0f ? -loT : __builtin_inff();
    const float th = hiT > 0.0f ? -hiT : __builtin_inff();
    const float qnan = __builtin_nanf("");
    f4 *stage = sStage[w];
    int scnt = 0; // staged entries of this wave
    if (tid == 0) sCnt = 0;
    if (sc.bpart)
        for (int e = tid; e < NBK; e += 256) sBk[e] = 0;
    __syncthreads();

    uint64_t *region = sc.region + (int64_t)blockIdx.x * sc.cap;
    // scalar, 64-bit: one wave may classify more than 2^32 pairs (a small
    // collect grid, or large N at d > 16)
    unsigned long long below = 0;
    const int xl = 4 * kq - ql; // j - i = xl + r + 16 (w - rb) on diagonal tiles

    // staged entries -> keys (s = max(-v, 0), as k_pair_tiles' fmax) in the
    // block's region (one LDS atomic per value slot and 64 entries) and the
    // bucket histogram
    auto flush = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); // other lanes' staging stores
        for (int q0 = 0; q0 < scnt; q0 += 64) {
            const f4 e = q0 + lane < scnt ? stage[q0 + lane] : f4{qnan, qnan, qnan, qnan};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float v = e[r];
                const bool keep = v == v;
                const unsigned long long mk = __ballot(keep);
                if (!mk) continue;
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(&sCnt, (uint32_t)__popcll(mk));
                base = __shfl(base, 0);
                if (keep) {
                    const uint64_t key = key_of((double)(v >= 0.0f ? 0.0f : -v));
                    const int64_t pos = (int64_t)base + __popcll(mk & ((1ull << lane) - 1ull));
                    if (pos < sc.cap) region[pos] = key;
                    if (sc.bpart) atomicAdd(&sBk[kbucket(key, lo_key, binv)], 1u);
                }
            }
        }
        scnt = 0;
        __builtin_amdgcn_s_waitcnt(0xF70); // vmcnt(0): the flush's stores drained here, once (see the column loop)
    };

    struct Cols {
        uint4 A3[NDB][3];
        f4 nv;    // norms of columns j0 + 4 kq + r (plain lane map)
        float nq; // norm of column j0 + ql (transposed lane map)
    };
    auto load_cols = [&](int J, Cols &c) {
        const int64_t j0 = (int64_t)J * TB + 16 * w;
        const uint4 *p = reinterpret_cast<const uint4 *>(xk + ((int64_t)J * 4 + w) * kb3_block_words(KP)) + lane;
#pragma unroll
        for (int db = 0; db < NDB; ++db)
#pragma unroll
            for (int q = 0; q < 3; ++q) c.A3[db][q] = p[(db * 3 + q) * 64];
        c.nv = *reinterpret_cast<const f4 *>(nrm + j0 + 4 * kq);
        c.nq = nrm[j0 + ql];
    };

    // the tile row's 4 row blocks' parts and norms, in VGPRs for the whole
    // run of tiles that share the row (~nb / 2): no LDS reads per tile
    uint4 rp[4][NDB][3];
    float hr[4]; // -n_i of row 16 rb + ql (plain lane map)
    f4 hn[4];    // -n_i of rows 16 rb + 4 kq + r (transposed lane map)
    auto rows = [&](int I) {
        const int ib = I * TB;
        const uint4 *src = reinterpret_cast<const uint4 *>(xk + (int64_t)I * 4 * kb3_block_words(KP)) + lane;
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
#pragma unroll
            for (int db = 0; db < NDB; ++db)
#pragma unroll
                for (int q = 0; q < 3; ++q) rp[rb][db][q] = src[((rb * NDB + db) * 3 + q) * 64];
            hr[rb] = -nrm[ib + 16 * rb + ql];
            hn[rb] = -*reinterpret_cast<const f4 *>(nrm + ib + 16 * rb + 4 * kq);
        }
        __builtin_amdgcn_s_waitcnt(0x0F70); // (vmcnt(0): the waits in the loop cover one column buffer)
    };

    // one tile of a kind: SW = wrapped (rows in the A role), DG = diagonal
    auto tile = [&](auto sw_tag, auto dg_tag, const Cols &c) {
        constexpr bool SW = decltype(sw_tag)::value, DG = decltype(dg_tag)::value;
        f4 acc[4];
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) acc[rb] = f4{0.0f, 0.0f, 0.0f, 0.0f};
        // term by term across the 4 row blocks' chains (each chain keeps the
        // key's order: tm, then db)
#pragma unroll
        for (int tm = 0; tm < 6; ++tm)
#pragma unroll
            for (int db = 0; db < NDB; ++db)
#pragma unroll
                for (int rb = 0; rb < 4; ++rb)
                    acc[rb] = SW ? kb3_mfma(rp[rb][db][KB3_TA[tm]], c.A3[db][KB3_TB[tm]], acc[rb])
                                 : kb3_mfma(c.A3[db][KB3_TA[tm]], rp[rb][db][KB3_TB[tm]], acc[rb]);
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
            // (-n_i) + (-n_j), packed, then v = fma(2, dot, .) (v_pk_fma_f32)
            typedef float f2 __attribute__((ext_vector_type(2)));
            const f2 two = {2.0f, 2.0f};
            f2 t01, t23;
            if constexpr (SW) { // row 16 rb + 4 kq + r, column ql
                const f2 qq = {-c.nq, -c.nq};
                t01 = f2{hn[rb][0], hn[rb][1]} + qq;
                t23 = f2{hn[rb][2], hn[rb][3]} + qq;
            } else {
                const f2 hh = {hr[rb], hr[rb]};
                t01 = hh + f2{-c.nv[0], -c.nv[1]};
                t23 = hh + f2{-c.nv[2], -c.nv[3]};
            }
            const f2 v01 = __builtin_elementwise_fma(two, f2{acc[rb][0], acc[rb][1]}, t01);
            const f2 v23 = __builtin_elementwise_fma(two, f2{acc[rb][2], acc[rb][3]}, t23);
            const f4 v = {v01[0], v01[1], v23[0], v23[1]};
            unsigned long long h[4], any = 0;
            uint32_t nbl = 0;
            if constexpr (DG) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    h[r] = mcol_classify_diag(v[r], tl, th, xl, 16 * rb - 16 * w - r, nbl);
                    any |= h[r];
                }
            } else {
                any = mcol_classify4(v, tl, th, nbl, h);
            }
            below += nbl;
            // band values (~1 % of the pairs): one entry per lane holding any
            if (__builtin_expect(any != 0, 0)) {
                const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(any >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)any, 0u));
                const f4 e = {lane_sel(h[0], v[0], qnan), lane_sel(h[1], v[1], qnan),
                              lane_sel(h[2], v[2], qnan), lane_sel(h[3], v[3], qnan)};
                // every lane stores: lanes without band values into the spill zone
                stage[lane_bit(any) ? scnt + (int)pre : TC3_ENT + lane] = e;
                scnt += __popcll(any);
            }
        }
    };

    // Per row: its parts, then its slots two at a time over two column
    // buffers; the next tile's columns load during the current tile's MFMAs
    // (block 0 when there is none, so the wait never includes it)
    const TileSched ts(nb, t0, t1);
    TileSched::Pos p0 = ts.first();
    auto run = [&](const TileSched::Pos &p, const Cols &c) {
        if (scnt > TC3_ENT - 256) flush(); // (one call site: the tile kinds share it)
        if (p.s == 0)
            tile(std::false_type{}, std::true_type{}, c);
        else if (p.J < p.I)
            tile(std::true_type{}, std::false_type{}, c);
        else
            tile(std::false_type{}, std::false_type{}, c);
    };
    if (ts.enter_row(p0)) {
        Cols c0, c1;
        load_cols(p0.J, c0);
        for (bool live = true; live;) {
            rows(p0.I);
            for (;;) {
                TileSched::Pos p1 = p0;
                const bool m1 = ts.advance(p1);
                load_cols(m1 ? p1.J : 0, c1);
                __builtin_amdgcn_sched_barrier(0); // the prefetch issues before the MFMAs
                run(p0, c0);
                if (!m1) {
                    live = false;
                    break;
                }
                if (p1.I != p0.I) { // next row: its first columns are in c1
                    p0 = p1;
                    c0 = c1;
                    break;
                }
                TileSched::Pos p2 = p1;
                const bool m2 = ts.advance(p2);
                load_cols(m2 ? p2.J : 0, c0);
                __builtin_amdgcn_sched_barrier(0);
                run(p1, c1);
                if (!m2) {
                    live = false;
                    break;
                }
                const bool row_end = p2.I != p1.I;
                p0 = p2;
                if (row_end) break;
            }
        }
    }

    if (scnt) flush();
    if (lane == 0) sBelow[w] = below;
    __syncthreads();
    if (tid == 0) {
        sc.below_out[blockIdx.x] = sBelow[0] + sBelow[1] + sBelow[2] + sBelow[3];
        sc.count_out[blockIdx.x] = sCnt;
    }
    if (sc.bpart)
        for (int e = tid; e < NBK; e += 256) sc.bpart[(int64_t)blockIdx.x * NBK + e] = sBk[e];
}


// ============================================================ launcher ==

#define SVGD_TCOL_CASE(KPv)                                                                  \
    case KPv:                                                                                \
        hipLaunchKernelGGL((k_pair_tcol<KPv>), dim3(grid), dim3(256), 0, stream, xc, nrm, n, nb, \
                           t0, t1, sc);                                                      \
        break;
#define SVGD_TCOL3_CASE(KPv)                                                                 \
    case KPv:                                                                                \
        hipLaunchKernelGGL((k_pair_tcol3<KPv>), dim3(grid), dim3(256), 0, stream, nrm, xk, n, nb, \
                           t0, t1, sc);                                                      \
        break;

hipError_t launch_pair_tcol(int KP, int grid, const float *xc, const float *nrm, const uint32_t *xk,
                            int64_t n, int64_t nb, int64_t t0, int64_t t1, uint64_t *regions,
                            int64_t cap, uint32_t *counts, unsigned long long *below,
                            const SelState *st, uint32_t *bpart, hipStream_t stream)
{
    if (grid <= 0 || t1 <= t0) return hipSuccess;
    if (kb3_keys(KP) && !xk) return hipErrorInvalidValue;
    SinkCollect sc{st, regions, cap, counts, below, nullptr, nullptr, bpart};
    switch (KP) {
        SVGD_TCOL_CASE(4)
        SVGD_TCOL_CASE(8)
        SVGD_TCOL_CASE(12)
        SVGD_TCOL_CASE(16)
        SVGD_TCOL3_CASE(32)
        SVGD_TCOL3_CASE(64)
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

#define SVGD_MCOL_CASE(Dv)                                                                   \
    case Dv:                                                                                 \
        hipLaunchKernelGGL((k_pair_mcol<Dv>), dim3(grid), dim3(256), 0, stream, xc, xf, xs, n, nb, \
                           t0, t1, sc);                                                      \
        break;
#define SVGD_MCOLB_CASE(Dv)                                                                  \
    case Dv:                                                                                 \
        hipLaunchKernelGGL((k_pair_mcol<Dv, true>), dim3(grid), dim3(256), 0, stream, xc, xf, xs, n, \
                           nb, t0, t1, sc);                                                  \
        return hipGetLastError();


hipError_t launch_pair_mcol(int d, int grid, const double *xc, const float *xf,
                            const unsigned long long *nmax_bits, int64_t n, int64_t nb, int64_t t0,
                            int64_t t1, uint64_t *regions, int64_t cap, uint32_t *counts,
                            unsigned long long *below, const SelState *st, uint32_t *bpart,
                            const uint32_t *xsplit, hipStream_t stream)
{
    if (grid <= 0 || t1 <= t0) return hipSuccess;
    if (!nmax_bits || !xf) return hipErrorInvalidValue;
    SinkCollect sc{st, regions, cap, counts, below, xf, nmax_bits, bpart};
    const uint4 *xs = reinterpret_cast<const uint4 *>(xsplit);
    if (d <= 8 && xs) { // the bf16-split Gram (k_pair_mcol<D, true>)
        switch (d) {
            SVGD_MCOLB_CASE(1)
            SVGD_MCOLB_CASE(2)
            SVGD_MCOLB_CASE(3)
            SVGD_MCOLB_CASE(4)
            SVGD_MCOLB_CASE(5)
            SVGD_MCOLB_CASE(6)
            SVGD_MCOLB_CASE(7)
            SVGD_MCOLB_CASE(8)
        default:
            break;
        }
    }
    switch (d) {
        SVGD_MCOL_CASE(1)
        SVGD_MCOL_CASE(2)
        SVGD_MCOL_CASE(3)
        SVGD_MCOL_CASE(4)
        SVGD_MCOL_CASE(5)
        SVGD_MCOL_CASE(6)
        SVGD_MCOL_CASE(7)
        SVGD_MCOL_CASE(8)
        SVGD_MCOL_CASE(9)
        SVGD_MCOL_CASE(10)
        SVGD_MCOL_CASE(11)
        SVGD_MCOL_CASE(12)
        SVGD_MCOL_CASE(13)
        SVGD_MCOL_CASE(14)
        SVGD_MCOL_CASE(15)
        SVGD_MCOL_CASE(16)
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

} // namespace svgd_amd
