// plan.cpp -- host-only work partitioning of the SVGD step (no GPU needed).
//
// Rows: particle i's phi_hat (SVGD.hpp:407-454) depends on every particle
// but is written only to row i, and the optimizer state is per particle
// (Adam.hpp:61-67), so ranks own contiguous row ranges.
//
// Median pairs: the reference takes the median over all n^2 distances
// (GaussianRBFKernel.hpp:185, 222-254): n diagonal zeros plus every
// off-diagonal distance twice.  Only the n(n-1)/2 upper-triangle values are
// visited, as block x block tiles (block = 256 on the row-stream path, 64 on
// the MFMA tile path): row block I pairs with itself (upper
// triangle inside the tile) and with column blocks I+1 .. I+H (mod nb),
// H = floor((nb-1)/2), plus I + nb/2 when nb is even and I < nb/2.  Every
// unordered pair of blocks then appears exactly once and every row block
// has the same number of tiles (+-1), so contiguous tile ranges balance the
// ranks.
#include <limits.h>
#include <stdint.h>

#include "../../include/svgdcpp_amd/svgd_capi.h"

extern "C" {

// Equal chunks of ceil(n/world) rows (the last ones may be short or empty),
// so the per-step all-gather is a single in-place ncclAllGather.
void svgd_plan_rows(int64_t n, int world, int rank, int64_t *row0, int64_t *row1)
{
    if (world < 1) world = 1;
    const int64_t chunk = (n + world - 1) / world;
    const int64_t r0 = chunk * rank, r1 = chunk * (rank + 1);
    *row0 = r0 < n ? r0 : n;
    *row1 = r1 < n ? r1 : n;
}

int svgd_plan_median_ranks(int64_t n, int64_t *rank_lo, int64_t *rank_hi)
{
    // full sorted list v of n^2 values; index k < n are the diagonal zeros,
    // index k >= n maps to upper-list rank (k - n) / 2.
    const int64_t total = n * n;
    auto map = [n](int64_t k) -> int64_t { return k < n ? -1 : (k - n) / 2; };
    if (total % 2 == 0) {
        *rank_lo = map(total / 2 - 1);
        *rank_hi = map(total / 2);
        return 2;
    }
    *rank_lo = *rank_hi = map(total / 2);
    return 1;
}

static int64_t tiles_total(int64_t nb) { return nb * (nb + 1) / 2; }

int64_t svgd_plan_pair_tiles(int64_t n, int block, int world, int rank)
{
    const int64_t nb = (n + block - 1) / block;
    const int64_t T = tiles_total(nb);
    if (world < 1) world = 1;
    return T * (rank + 1) / world - T * rank / world;
}

void svgd_plan_pair_tile(int64_t n, int block, int world, int rank, int64_t t,
                         int64_t *row_block, int64_t *col_block)
{
    const int64_t nb = (n + block - 1) / block;
    if (world < 1) world = 1;
    t += tiles_total(nb) * rank / world;
    const int64_t H = (nb - 1) / 2;
    int64_t I, slot;
    if ((nb & 1) == 0) {
        const int64_t c1 = H + 2, c2 = H + 1, half = nb / 2;
        if (t < half * c1) {
            I = t / c1;
            slot = t - I * c1;
        } else {
            const int64_t u = t - half * c1;
            I = half + u / c2;
            slot = u - (I - half) * c2;
        }
    } else {
        I = t / (H + 1);
        slot = t - I * (H + 1);
    }
    *row_block = I;
    *col_block = slot == 0 ? I : (I + slot) % nb;
}

// The symmetric phi pass's units: (tile, sub-tile) pairs of the tile plan in
// order, each tile's sub-tiles of `block / nsub` columns -- except the last
// column block's sub-tiles past n (all padding columns), which are not units
// at all: at N = 2^16 and 2^18 with 1536-row blocks the real units then
// divide evenly over 256 work-groups at P = 1, 2, 4 and 8.
static int64_t sym_cnt_h(int64_t nb, int64_t I) // tiles of row block I (slots 0 .. cnt-1)
{
    const int64_t H = (nb - 1) / 2;
    return ((nb & 1) == 0 && I < nb / 2) ? H + 2 : H + 1;
}
static int64_t sym_qlast(int64_t n, int block, int nsub, int64_t nb) // real sub-tiles of block nb - 1
{
    const int64_t sub = block / nsub, valid = n - (nb - 1) * block;
    return (valid + sub - 1) / sub;
}
// units of row block I: its tiles' sub-tiles, the one tile (if any) whose
// column block is the last one counting qlast
static int64_t sym_units_of(int64_t nb, int nsub, int64_t qlast, int64_t I)
{
    const int64_t cnt = sym_cnt_h(nb, I), s = nb - 1 - I; // slot of column block nb - 1
    return cnt * nsub - (s < cnt ? nsub - qlast : 0);
}

int64_t svgd_plan_sym_total(int64_t n, int block, int nsub)
{
    const int64_t nb = (n + block - 1) / block, ql = sym_qlast(n, block, nsub, nb);
    int64_t U = 0;
    for (int64_t I = 0; I < nb; ++I) U += sym_units_of(nb, nsub, ql, I);
    return U;
}

int svgd_plan_sym_unit(int64_t n, int block, int nsub, int64_t u, int64_t *tile, int64_t *q)
{
    const int64_t nb = (n + block - 1) / block, ql = sym_qlast(n, block, nsub, nb);
    int64_t t = 0;
    for (int64_t I = 0; I < nb; ++I) {
        const int64_t uI = sym_units_of(nb, nsub, ql, I), cnt = sym_cnt_h(nb, I);
        if (u >= uI) {
            u -= uI;
            t += cnt;
            continue;
        }
        for (int64_t slot = 0; slot < cnt; ++slot) {
            const int64_t J = (I + slot) % nb, nq = J == nb - 1 ? ql : nsub;
            if (u < nq) {
                *tile = t + slot;
                *q = u;
                return 0;
            }
            u -= nq;
        }
    }
    *tile = *q = -1;
    return -1;
}

// The symmetric phi pass's unit plan (svgd_capi.cpp, k_phi_sym / k_sym_finish).
int64_t svgd_plan_sym_units(int64_t n, int block, int nsub, int world, int rank, int grid,
                            int64_t *u0, int64_t *u1, int *blkg, int *rbase, int64_t *Ia, int64_t *Ib)
{
    if (world < 1) world = 1;
    const int64_t nb = (n + block - 1) / block;
    const int64_t U = svgd_plan_sym_total(n, block, nsub);
    *u0 = U * rank / world;
    *u1 = U * (rank + 1) / world;
    const int64_t V = *u1 - *u0;
    for (int64_t P = 0; P < nb; ++P) {
        blkg[2 * P] = INT32_MAX;
        blkg[2 * P + 1] = -1;
    }
    *Ia = 0;
    *Ib = -1;
    if (V <= 0 || grid < 1) {
        for (int64_t P = 0; P < nb; ++P) rbase[P] = 0;
        return 0;
    }
    // work-group g takes the contiguous units [u0 + V g / G, u0 + V (g+1) / G)
    // (G <= V: none is empty) and visits the row blocks of their tiles
    int64_t J;
    for (int64_t g = 0; g < grid; ++g) {
        const int64_t a = *u0 + V * g / grid, b = *u0 + V * (g + 1) / grid;
        if (b <= a) continue;
        int64_t I0, I1, ta, tb, q;
        svgd_plan_sym_unit(n, block, nsub, a, &ta, &q);
        svgd_plan_sym_unit(n, block, nsub, b - 1, &tb, &q);
        svgd_plan_pair_tile(n, block, 1, 0, ta, &I0, &J);
        svgd_plan_pair_tile(n, block, 1, 0, tb, &I1, &J);
        for (int64_t P = I0; P <= I1; ++P) {
            if ((int)g < blkg[2 * P]) blkg[2 * P] = (int)g;
            if ((int)g > blkg[2 * P + 1]) blkg[2 * P + 1] = (int)g;
        }
    }
    // each row block's row-sum records contiguous, in work-group order
    int64_t nrec = 0;
    for (int64_t P = 0; P < nb; ++P) {
        rbase[P] = (int)nrec;
        if (blkg[2 * P + 1] >= blkg[2 * P]) nrec += blkg[2 * P + 1] - blkg[2 * P] + 1;
    }
    int64_t ta, tb, q;
    svgd_plan_sym_unit(n, block, nsub, *u0, &ta, &q);
    svgd_plan_sym_unit(n, block, nsub, *u1 - 1, &tb, &q);
    svgd_plan_pair_tile(n, block, 1, 0, ta, Ia, &J);
    svgd_plan_pair_tile(n, block, 1, 0, tb, Ib, &J);
    return nrec;
}

// The particles rank src's symmetric-pass units add to: a cyclic run of
// blocks from its first row block Ia through Ib + the largest slot (SM - 1 =
// (nb - 1) / 2 + 1, the even-nb extra slot included: a hull), intersected
// with dst's rows.
void svgd_plan_sym_exchange(int64_t n, int block, int nsub, int world, int src, int dst, int64_t *r0,
                            int64_t *r1)
{
    if (world < 1) world = 1;
    int64_t d0, d1;
    svgd_plan_rows(n, world, dst, &d0, &d1);
    *r0 = *r1 = d0;
    const int64_t nb = (n + block - 1) / block;
    const int64_t U = svgd_plan_sym_total(n, block, nsub);
    const int64_t u0 = U * src / world, u1 = U * (src + 1) / world;
    if (u1 <= u0 || d1 <= d0) return;
    int64_t Ia, Ib, J, ta, tb, q;
    svgd_plan_sym_unit(n, block, nsub, u0, &ta, &q);
    svgd_plan_sym_unit(n, block, nsub, u1 - 1, &tb, &q);
    svgd_plan_pair_tile(n, block, 1, 0, ta, &Ia, &J);
    svgd_plan_pair_tile(n, block, 1, 0, tb, &Ib, &J);
    const int64_t len = Ib - Ia + 1 + (nb - 1) / 2 + 1; // blocks Ia .. Ib + SM - 1
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    auto meet = [&](int64_t a, int64_t b) { // particles [a, b) against dst's rows
        a = a > d0 ? a : d0;
        b = b < d1 ? b : d1;
        if (a < b) {
            lo = a < lo ? a : lo;
            hi = b > hi ? b : hi;
        }
    };
    if (len >= nb) {
        meet(0, n);
    } else if (Ia + len <= nb) {
        meet(Ia * block, (Ia + len) * block < n ? (Ia + len) * block : n);
    } else {
        meet(Ia * block, n);
        meet(0, (Ia + len - nb) * block);
    }
    if (lo < hi) {
        *r0 = lo;
        *r1 = hi;
    }
}

// Bucket of each selection from the all-reduced key-range bucket counts
// (NBK buckets, ascending key order): ranks[s] is the rank among the
// candidates; writes the bucket and the rank within it, and the total count
// of the distinct selected buckets.  Returns -1 if a rank lies past the
// counted candidates.
int svgd_plan_bucket_select(const unsigned long long *counts, int nb, int nsel,
                            const int64_t *ranks, int *bsel, int64_t *rank_in, int64_t *total)
{
    if (nsel < 1 || nsel > 2) return -1;
    int64_t cum = 0;
    bsel[0] = bsel[1] = -1;
    for (int b = 0; b < nb; ++b) {
        const int64_t c = (int64_t)counts[b];
        for (int s = 0; s < nsel; ++s)
            if (bsel[s] < 0 && ranks[s] >= cum && ranks[s] < cum + c) {
                bsel[s] = b;
                rank_in[s] = ranks[s] - cum;
            }
        cum += c;
    }
    for (int s = 0; s < nsel; ++s)
        if (bsel[s] < 0) return -1;
    if (nsel == 1) {
        bsel[1] = bsel[0];
        rank_in[1] = rank_in[0];
    }
    *total = (int64_t)counts[bsel[0]] + (bsel[1] != bsel[0] ? (int64_t)counts[bsel[1]] : 0);
    return 0;
}

} // extern "C"
