// svgd_device.h -- device helpers shared by the gfx950 kernel translation
// units (svgd_kernels.hip, svgd_collect.hip).  Internal.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "svgd_kernels.h"

namespace svgd_amd {

typedef float f4_t __attribute__((ext_vector_type(4)));

constexpr int PBLK = 256; // row/column block of the row-stream median tile plan (plan.cpp)
constexpr int TB = 64;    // particles per tile of the MFMA tile kernels (rows and columns)

// Coordinate k taken by MFMA step kk and lane group q (= lane / 16) in the
// pair-key Gram of the tile kernels (k_pair_tiles, k_pair_tcol; every pass
// over the keys uses the same order, so they agree bit for bit).  fp32 with
// KP % 16 == 0: the steps 4u..4u+3 of lane group q read coordinates
// 16u + 4q .. 16u + 4q + 3, i.e. one 16-byte load per 4 steps and 64
// contiguous bytes per row for the 4 groups; otherwise 4 kk + q.
template <class T, int KP> __device__ __forceinline__ constexpr int kslot(int kk, int q)
{
    if constexpr (sizeof(T) == 4 && KP % 16 == 0)
        return 16 * (kk >> 2) + 4 * q + (kk & 3);
    else
        return 4 * kk + q;
}

// --------------------------------------------------------------- median --

// The split-bf16 form of 8 fp32 coordinates (k_pair_mcol<D, true>'s Gram):
// x = hi + lo + r, hi = bf16(x), lo = bf16(x - hi) (x - hi exact in fp32),
// |r| <= 2^-16 |x|; lo_part selects which half (8 bf16 = 16 bytes).  Written
// once per particle and step by the centring (k_center_d, xs), read by the
// collect as its A and B fragments.
__device__ __forceinline__ uint4 mcol_split_bf16(const float (&x)[8], bool lo_part)
{
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const __hip_bfloat162 h = __float22bfloat162_rn(make_float2(x[2 * q], x[2 * q + 1]));
        const uint32_t hb = *reinterpret_cast<const uint32_t *>(&h);
        const float r0 = x[2 * q] - __uint_as_float(hb << 16);
        const float r1 = x[2 * q + 1] - __uint_as_float(hb & 0xffff0000u);
        const __hip_bfloat162 l = __float22bfloat162_rn(make_float2(r0, r1));
        const uint32_t lb = *reinterpret_cast<const uint32_t *>(&l);
        o[q] = lo_part ? lb : hb;
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}
//
// Keys: squared distances s = max((|xc_i|^2 + |xc_j|^2) - 2 xc_i.xc_j, 0)
// (the reference's Gram form, GaussianRBFKernel.hpp:179-183, on centred
// coordinates) as the IEEE bit pattern, which orders like uint64 for s >= 0.
// Every unordered pair i<j is visited once by the tile sweep of plan.h.

__device__ __forceinline__ uint64_t key_of(double s)
{
    return (uint64_t)__double_as_longlong(s) & 0x7fffffffffffffffull; // s >= 0 (+0, never -0)
}

// Key-range bucket of a candidate key (SelState::binv): monotone in the key.
__device__ __forceinline__ int kbucket(uint64_t key, uint64_t lo, double binv)
{
    const double t = (double)(key - lo) * binv;
    return t < (double)(NBK - 1) ? (t > 0.0 ? (int)t : 0) : NBK - 1;
}

// Device copy of plan_pair_tile (plan.cpp): tile index -> (row block, col block).
__device__ __forceinline__ void tile_coords(int64_t nb, int64_t t, int64_t *I, int64_t *J)
{
    const int64_t H = (nb - 1) / 2;
    int64_t slot;
    if ((nb & 1) == 0) {
        const int64_t c1 = H + 2, c2 = H + 1, half = nb / 2;
        if (t < half * c1) {
            *I = t / c1;
            slot = t - *I * c1;
        } else {
            const int64_t u = t - half * c1;
            *I = half + u / c2;
            slot = u - (*I - half) * c2;
        }
    } else {
        const int64_t c = H + 1;
        *I = t / c;
        slot = t - *I * c;
    }
    *J = slot == 0 ? *I : (*I + slot) % nb;
}

// ------------------------------------------ F32 pair keys for d > 16 (B3) --
//
// SVGD_F32 with KP in {32, 64}: the Gram of every pair key is formed on the
// bf16 matrix cores (16x the fp32 MFMA rate) from the exact three-part bf16
// split of the fp32 centred coordinates, x = h + m + l, with the six part
// products that reach 2^-24 of each product (as k_phi_b3).  The key of a
// pair i < j is DEFINED by this sequence, and every pass over the keys (the
// matrix-core collect k_pair_tcol, k_pair_tiles' collect / radix / debug /
// sample modes) runs it, so they agree bit for bit:
//   dot = 0; for tm = 0..5 (mm, hl, lh, hm, mh, hh), for db = 0..KP/32 - 1:
//     dot = v_mfma_f32_16x16x32_bf16(A = part KB3_TA[tm] of x_j, k-chunk db,
//                                    B = part KB3_TB[tm] of x_i, k-chunk db, dot)
//   s = max(fma(-2, dot, n_i + n_j), 0)
// with x_j the particle of the LARGER index: the hm / mh terms are not
// symmetric under the swap of the operand roles, so a tile whose column
// block precedes its row block (the plan's wrapped tiles) swaps them.
// Parts (k_swz_keys_b3, once per step from xcf), per 16-row block b:
//   XK[b][db][part][lane][e] = part of xcf[16 b + lane % 16][32 db + 8 (lane / 16) + e]
// (the A and B operand lane maps of the 16x16x32 MFMA coincide).
constexpr int KB3_TA[6] = {1, 0, 2, 0, 1, 0}, KB3_TB[6] = {1, 2, 0, 1, 0, 0};
__host__ __device__ constexpr bool kb3_keys(int KP) { return KP == 32 || KP == 64; }
__host__ __device__ constexpr int kb3_block_words(int KP) { return (KP / 32) * 3 * 256; }
typedef __bf16 kb3_bf16x8_t __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f4_t kb3_mfma(uint4 a, uint4 b, f4_t c)
{
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(kb3_bf16x8_t, a),
                                                   __builtin_bit_cast(kb3_bf16x8_t, b), c, 0, 0, 0);
}
// One 16 x 16 block of dots from the parts in memory (global or LDS): pa =
// the larger-index block's parts, pb = the other's, each at + lane * 4.
template <int KP> __device__ __forceinline__ f4_t kb3_dot(const uint32_t *pa, const uint32_t *pb)
{
    constexpr int NDB = KP / 32;
    uint4 a[NDB][3], b[NDB][3];
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            a[db][p] = *reinterpret_cast<const uint4 *>(pa + (db * 3 + p) * 256);
            b[db][p] = *reinterpret_cast<const uint4 *>(pb + (db * 3 + p) * 256);
        }
    f4_t dot = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int tm = 0; tm < 6; ++tm)
#pragma unroll
        for (int db = 0; db < NDB; ++db) dot = kb3_mfma(a[db][KB3_TA[tm]], b[db][KB3_TB[tm]], dot);
    return dot;
}

struct SinkCollect {
    const SelState *st; // bracket [st->lo_key, st->hi_key)
    uint64_t *region; // this block's region (capacity cap)
    int64_t cap;
    uint32_t *count_out;
    unsigned long long *below_out;
    const float *xf;                     // fp32 records (unused by the collect pass)
    const unsigned long long *nmax_bits; // max |xc|^2 (double bits): classification margin
    uint32_t *bpart;                     // per-block key-range bucket histograms (optional)
};

struct SinkHist {
    const SelState *st;
    unsigned long long *ghist; // [2][RADIX] (64-bit: a streamed pass counts up to n(n-1)/2 keys)
};

struct SinkDebug {
    double *out;    // MODE 2: every upper-triangle distance at its list index
    int64_t n;
    uint64_t *keys; // MODE 3: 64 x 64 keys of each sampled tile
};

} // namespace svgd_amd
