// svgd_kernels.h -- host-callable launchers of the gfx950 kernels (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace svgd_amd {

constexpr int RADIX_BITS = 11;
constexpr int RADIX = 1 << RADIX_BITS;

// Device-resident state of the (dual) radix select over 63-bit keys
// (non-negative doubles as uint64).  Digits from the top: bits 62..52,
// 51..41, 40..30, 29..19, 18..8, 7..0.
struct SelState {
    uint64_t prefix[2];   // resolved high bits of the two selected keys
    uint64_t rank[2];     // remaining rank within the current prefix
    uint64_t lo_key;      // candidate bracket [lo_key, hi_key)
    uint64_t hi_key;
    int32_t nsel;         // 1 or 2 active selections
    int32_t shift;        // shift of the current digit
    int32_t width;        // width of the current digit
    int32_t pass;         // digits resolved so far
    int32_t error;        // rank outside the histogram (should not happen)
    int32_t pad_;
    double binv;          // key-range buckets of [lo_key, hi_key): NBK / (hi - lo)
    int32_t bsel[2];      // bucket of each selection (bucket select path)
};

// Key-range buckets of the candidate bracket: bucket(key) = floor((key - lo)
// * binv), clamped to [0, NBK) -- monotone in the key, so buckets are
// contiguous key ranges.  The collect pass histograms them, so one all-reduce
// (counts + buckets) tells every rank which bucket holds each order statistic.
constexpr int NBK = 2048;
// per-rank capacity of the compacted selected-bucket keys (gathered over
// ranks).  At cfg4 (N = 262144, 3.4e10 pairs) a sampled bracket's bucket
// holds ~25k keys on one rank (2^22-pair sample) and ~100k at P > 1 (2^20):
// 16384 sent every cfg4 step down the radix path, so it never speculated
// and never tracked its bracket.  The synchronous path's all-gather moves
// the step's own total, the speculative one the adaptive spec cap.
constexpr int CAPG = 262144;

// xc = X - mu (stride KP, zero padded), nrm = |xc|^2; nrm_in_slot also
// stores |xc|^2 at xc[j*KP + d] (the row-stream median record).
// xf (optional, d <= 16): fp32 median records [xc | -|xc|^2/2 | 0..] of stride
// med_f32_stride(d); nmax_bits: max |xc|^2 as double bits (atomicMax).
// bzero (optional): NBK counters zeroed (the step's collect-pass bucket counts)
// st_init (optional): written to *st_out by the launch (a predicted bracket)
// The centre mu: the exact mean of X (k_mean_partial into partial[nparts],
// which also zeroes nmax_bits), or -- the fold, d <= 16 on the row path, one
// launch -- the mean of another X from its column partials pin[nin] (the
// ones a previous centring left: the previous particles' mean).  Row path:
// pout (optional) <- this X's column partials (center_fold_grid(d, np)
// blocks of d) and *nmax_zero = 0 (the next centring's max target).
int center_fold_grid(int d, int64_t np);
hipError_t launch_mean_center(const double *X, int64_t n, int d, int KP, int64_t np,
                              double *partial, int nparts, double *xc, double *nrm,
                              int nrm_in_slot, float *xf, unsigned long long *nmax_bits,
                              unsigned long long *bzero, hipStream_t stream,
                              SelState *st_out = nullptr, const SelState *st_init = nullptr,
                              const double *pin = nullptr, int nin = 0, double *pout = nullptr,
                              unsigned long long *nmax_zero = nullptr, float *xcf = nullptr,
                              float *nrmf = nullptr, uint32_t *xsplit = nullptr);
// (xcf / nrmf, KP 32 or 64: also the fp32 copies of xc and nrm, nrmf +inf in
// the padding rows -- launch_cvt_f32 / launch_cvt_nrm_f32 in the same pass;
// xsplit, d <= 8 with xf: the collect's split-bf16 operands, 8 dwords per
// particle [hi | lo] of its fp32 coordinates, rows [0, np))
hipError_t launch_prep_v(const double *xc, const double *G, const double *nrm, const double *a_ptr,
                         int64_t n, int64_t np, int d, int KP, int VW, double *V, double *cvec,
                         hipStream_t stream);
// n: particles (columns j >= n are padding); an fp64 tile with d = 16 NCB
// (phi_tile_s1v) sums P's rows on the VALU instead of a V column of ones
hipError_t launch_phi(int KP, int NCB, const double *xc, const double *cvec, const double *V,
                      const double *a_ptr, int64_t row0, int64_t nrows, int64_t ntiles_j, int64_t n,
                      int d, double inv_n, const double *wv, double *phi, hipStream_t stream);
bool phi_tile_s1v(int d);
void phi_tile_cfg(bool f64, int *nw, int *pre); // k_phi's waves per block and prefetch flag
// fp32 variants of the tile kernels (SVGD_F32); phi and the epilogue stay fp64
hipError_t launch_phi_f32(int KP, int NCB, const float *xg, const float *cvec, const float *V,
                          const double *a_ptr, int64_t row0, int64_t nrows, int64_t ntiles_j,
                          int64_t n, int d, double inv_n, const double *wv, const double *xc,
                          double *phi, hipStream_t stream);
hipError_t launch_pair_tiles_f32(int KP, int mode, int grid, const float *xc, const float *nrm,
                                 int64_t n, int64_t nb, int64_t t0, int64_t t1, uint64_t *regions,
                                 int64_t cap, uint32_t *counts, unsigned long long *below,
                                 const SelState *st, unsigned long long *ghist, uint32_t *bpart,
                                 double *dbg_out, const uint32_t *xk, hipStream_t stream);
hipError_t launch_cvt_f32(const double *src, int64_t cnt, float *dst, hipStream_t stream);
// fp32 copy of the norms with +inf in the padding rows [n, np)
hipError_t launch_cvt_nrm_f32(const double *src, int64_t n, int64_t np, float *dst, hipStream_t stream);
// Sampled median keys on the tile path: ntiles random (block, block) pairs of
// distinct full 64-particle blocks, all 64 x 64 keys each (xcf/nrmf: fp32 path)
// xk: the F32 key parts when KP is 32 or 64 (launch_swz_keys_b3), else null
hipError_t launch_sample_tiles(int KP, const double *xc, const double *nrm, const float *xcf,
                               const float *nrmf, const uint32_t *xk, int64_t n, int64_t ntiles,
                               uint64_t *keys, hipStream_t stream);
// The F32 median's key parts for KP = 32 / 64 (svgd_device.h "F32 pair keys"):
// np / 16 blocks of kb3_block_words(KP) dwords from xcf (stride KP); np % 16 == 0
hipError_t launch_swz_keys_b3(const float *xcf, int KP, int64_t np, uint32_t *XK, hipStream_t stream);
// dwords of those parts for np rows; 0 when the keys at this KP are the fp32-MFMA ones
int64_t median_key_part_words(int KP, int64_t np);
// bak (optional, 3 cnt doubles): X_t, m_t, v_t of the cnt elements, saved in the pass
// One optimizer step over cnt = rows x d elements of this rank (X, m, v at
// the rank's rows): Adam (kind 0) / AdaGrad (1) / RMSProp (2) + clamp.
struct OptArgs {
    int kind, d;
    int64_t cnt;
    double *m, *v, *X;
    double lr, b1, b2, eps, c1, c2;
    const double *lower, *upper; // clamp bounds (both or neither)
    double *bak;                 // X_t, m_t, v_t saved here when set (speculative step)
    double *xh = nullptr;        // X_{t+1} also stored here when set (pinned host mirror)
};
hipError_t launch_opt_update(const OptArgs &o, const double *g, hipStream_t stream);
// mode 0: collect keys in [st->lo_key, st->hi_key) into per-block regions and count
// keys below lo_key; mode 1: radix histogram pass over all pairs (fallback);
// mode 2: debug dump of every key in (i<j) row-major order.
// bpart (mode 0, optional): per-block key-range bucket histograms [grid][NBK]
hipError_t launch_pair_tiles(int KP, int mode, int grid, const double *xc, const double *nrm,
                             int64_t n, int64_t nb, int64_t t0, int64_t t1, uint64_t *regions,
                             int64_t cap, uint32_t *counts, unsigned long long *below,
                             const SelState *st, unsigned long long *ghist, uint32_t *bpart,
                             double *dbg_out, hipStream_t stream);
// xf != nullptr (d <= 16): keys from the fp32 records (a bracket estimate only).
// Sample pairs g0 .. g0+S-1 of the counter-based sequence -> keys[0 .. S-1]
// (ranks draw disjoint index ranges of one sequence).
// st_out (optional) <- init: the bracket passes' select state, set by the sampler.
hipError_t launch_sample_keys(const double *xc, const double *nrm, const float *xf, int64_t n,
                              int d, int KP, int64_t g0, int64_t S, uint64_t *keys,
                              const SelState &init, SelState *st_out, hipStream_t stream);
// ghist (2 RADIX u64) += this pass's digit histogram; zero on entry
hipError_t launch_hist_regions(const uint64_t *keys, const uint32_t *counts, int64_t nreg,
                               int64_t cap, int max_blocks, const SelState *st,
                               unsigned long long *ghist, hipStream_t stream);
hipError_t launch_compact(const uint64_t *keys, const uint32_t *counts, int64_t nreg, int64_t cap,
                          const SelState *st, uint64_t *cbuf, unsigned long long *ccount,
                          hipStream_t stream);
hipError_t launch_select_tail(SelState *st, const uint64_t *cbuf, const unsigned long long *ccount,
                              int passes, hipStream_t stream);
hipError_t launch_hist_count(const uint64_t *keys, const unsigned long long *ccount, int64_t cap,
                             const SelState *st, unsigned long long *ghist, hipStream_t stream);
// make_bracket: the sample's last pass also sets the candidate bracket (and
// zeroes bzero[0 .. NBK), the coming collect pass's bucket counts)
hipError_t launch_select_scan(SelState *st, unsigned long long *ghist, int make_bracket,
                              unsigned long long *bzero, hipStream_t stream);
// cnt = [below, candidates, overflowed regions, NBK bucket counts (zero without
// bpart), lo_key, hi_key]: the first 3 + NBK entries are sums over ranks.
constexpr int CNT_LO = 3 + NBK, CNT_HI = 4 + NBK, CNT_LEN = 5 + NBK;
hipError_t launch_counts_reduce(const unsigned long long *below, const uint32_t *counts,
                                int64_t nblk, int64_t cap, const SelState *st,
                                const uint32_t *bpart, int64_t nbpart,
                                unsigned long long *cnt, hipStream_t stream,
                                uint64_t *seg_zero = nullptr);
// (seg_zero, optional: zeroed -- the speculative compaction's counter)
// device state from kernel arguments (no host staging buffer)
hipError_t launch_set_state(const SelState &s, SelState *st, hipStream_t stream);
hipError_t launch_set_scal(double a, double med, double *scal, hipStream_t stream);
// bucket select path: the selections' ranks within their buckets (other fields
// kept) and a zeroed counter seg[0] for launch_compact_buckets
hipError_t launch_set_sel(SelState *st, int nsel, uint64_t r0, uint64_t r1, int b0, int b1,
                          uint64_t *seg, hipStream_t stream);
// keys of the selected buckets st->bsel[] -> seg = [count, keys (<= seg_cap)]
// (seg[0] must be zero on entry).  plan (optional, the speculative step):
// every block derives the bucket plan from the all-reduced counts itself
// (as launch_plan_select would) and block 0 publishes it (select state,
// *status, *host_status) -- one launch fewer per step.
struct PlanArgs {
    const unsigned long long *cnt; // nullptr: the plan is already in st
    int nsel;
    uint64_t r0, r1;
    int64_t capr;
    int *status, *host_status;
    // SVGD_SIM_WORLD measurement mode: one rank's share is selected alone, so
    // r0 is re-anchored at the middle of its candidates (r1 keeps r1 - r0)
    int sim = 0;
    // bracket tracking (optional, pinned host memory): [0] lo_key, [1] hi_key,
    // [2] below, [3] candidates of this step's bracket (block 0 of the plan)
    uint64_t *trk = nullptr;
};
hipError_t launch_compact_buckets(const uint64_t *keys, const uint32_t *counts, int64_t nreg,
                                  int64_t cap, SelState *st, uint64_t *seg, int64_t seg_cap,
                                  const int *status, hipStream_t stream,
                                  const PlanArgs *plan = nullptr);
// exact selection of st->rank[s] within bucket st->bsel[s] over nseg gathered
// segments [count, keys...] of stride seg_cap + 1 -> st->prefix[s] = that key,
// then the scale as launch_finalize
// trk (optional, pinned host memory): [4], [5] <- the selected keys, [6] <- error
hipError_t launch_select_small(SelState *st, const uint64_t *segs, int nseg, int64_t seg_cap,
                               int navg, int src_lo, int src_hi, double logn, double *scal,
                               const int *status, hipStream_t stream, uint64_t *trk = nullptr,
                               uint64_t seq = 0); // seq: stored into trk[8] at the end (spec steps)
// Device-side bucket plan from the all-reduced counts (speculative step): the
// select state, seg[0] = 0 and *status = 0, or *status = 1 (bracket miss),
// 2 (overflowed region), 3 (selected buckets hold > capr keys), also stored to
// host_status (device view of pinned host memory; optional).  The two
// launchers above do nothing unless *status == 0 (status nullptr: always run).
hipError_t launch_plan_select(const unsigned long long *cnt, SelState *st, int nsel, uint64_t r0,
                              uint64_t r1, int64_t capr, uint64_t *seg, int *status,
                              int *host_status, hipStream_t stream);
// per-rank segment capacity of the speculative bucket select: adaptive
// (svgd_capi.cpp plan_step: twice the last step's selected-bucket total,
// rounded up to a power of two, within [CAPR_MIN, CAPG]); the all-gather
// (P > 1) moves cap + 1 keys per rank.  At cfg3 a bucket holds ~3k keys:
// a fixed 4096 made ~1 in 5 early steps fail the plan (each failure redoes
// the step); the selection reads only the keys present.
constexpr int CAPR_MIN = 4096;

// Row-stream path (d <= 16): particle records rec_j = [xc_j | G_j - 2a xc_j | c_j | 0..],
// stride phi_rec_stride(d).  phi partials over S column splits -> part[S][ldp][d+1].
constexpr int ROWS_MAX_D = 16;
// record strides (doubles) of the row-stream path: phi records
// [xc | G - 2a xc | c | 0..] and median records [xc | |xc|^2 | 0..]
constexpr int phi_rec_stride(int d) { return ((2 * d + 1 + 7) / 8) * 8; }
constexpr int med_rec_stride(int d) { return ((d + 1 + 3) / 4) * 4; }
constexpr int med_f32_stride(int d) { return ((d + 1 + 7) / 8) * 8; }
hipError_t launch_prep_rec(const double *xc, const double *G, const double *nrm,
                           const double *a_ptr, int64_t n, int64_t np, int d, int KP, int RS,
                           double *rec, hipStream_t stream);
// opt (optional): the optimizer step applied to each phi element as the
// reduce writes it (the step path: one launch fewer than launch_opt_update).
// ev_mid (optional): recorded between k_phi_rows and its reduce (diagnostics).
hipError_t launch_phi_rows(int d, int R, const double *rec, const double *a_ptr,
                           int64_t row0, int64_t nrows, int64_t n, int S, double *part,
                           int64_t ldp, double inv_n, const double *wv, const double *sgn,
                           const unsigned long long *nmax_bits, double *phi, const OptArgs *opt,
                           hipStream_t stream, hipEvent_t ev_mid = nullptr, int kind = 0,
                           const int *skip = nullptr, bool reduce = true);
// skip (optional): the reduce does nothing while *skip != 0.  reduce = false:
// the row kernel alone

// Symmetric phi pass (d <= 8): each unordered pair's kernel value feeds both
// particles (k_phi_sym, launch_phi_sym), then k_sym_finish (launch_sym_finish)
// sums the partials in a fixed order, forms phi and applies the optimizer.
// The pair pass runs while *symok (set by its record prep: a log2e
// max|xc|^2 <= 300); otherwise the same launch runs the row stream's
// work-groups (its 8-wave kernel, fS column splits, on the rank's rows) and
// the finish (one rank) or k_sym_apply (P > 1) sums ITS partials fS x fldp
// (the k_phi_reduce arithmetic) -- no second launch on the usual path.
struct SymArgs {
    int d;
    const double *xc;
    int KP;
    const double *G, *nrm, *a_ptr;
    const unsigned long long *nmax;
    int64_t n, nbs, u0, u1; // particles, blocks of B, this rank's (tile, sub-tile) units [u0, u1)
    double *srec;          // nbs * B records of SRS doubles
    int *symok;
    double *rowpart;       // per row block P, its visiting work-groups' row sums (rbase below) x B x (d+1)
    double *colpart;       // nbs x SM slots x B x (d+1), by (column block, slot)
    int grid;
    int64_t row0, nrows;
    double inv_n;
    double *phi;
    double *rec; // the row stream's records, written by the record prep when symok = 0
    int RS;
    // P > 1: the finish writes every particle's sums from this rank's units
    // here (n x (d+1), the exchange's send buffer) instead of phi
    double *contrib = nullptr;
    // row-block tables: blkg[2P], blkg[2P+1] = the work-groups whose units
    // meet row block P (g1 < g0: none), rbase[P] = the first rowpart record of P
    const int *blkg = nullptr, *rbase = nullptr;
    int64_t SM = 0;        // colpart slots per column block: (nbs - 1) / 2 + 2
    int64_t Ia = 0, Ib = 0; // the row blocks this rank's units span
    // the row stream's partials when it takes the step (symok = 0)
    double *fpart = nullptr;
    int fS = 0;
    int64_t fldp = 0;
    // the first unit (tile, sub-tile) of each work-group's run
    // (svgd_plan_sym_unit) and the real sub-tiles of the last column block
    const int *wst = nullptr;
    int qlast = 0;
    const double *tab8k = nullptr; // the biased exp table (launch_fill_tab8k), 8192 doubles
};
hipError_t launch_fill_tab8k(double *tab, hipStream_t stream);
// P > 1: phi + the optimizer for rows [row0, row0 + nrows) from their sums:
// own (this rank's, nrows x (d+1)) and the pieces received from the other
// ranks (xtab: world x {t0, t1, row offset in recv}), added in rank order --
// or from the row stream's partials when symok = 0.  world = 1: own alone.
hipError_t launch_sym_apply(const SymArgs &a, const double *own, const double *recv, const int64_t *xtab,
                            int world, int rank, const OptArgs *opt, hipStream_t stream);
bool phi_sym_supported(int d);
bool phi_sym_geom(int d, int *B, int *SRS, int *NSUB);
int phi_sym_blocks_per_cu(int d);
// record prep + k_phi_sym (ev_k0 / ev_k1 around the pair kernel, optional)
hipError_t launch_phi_sym(const SymArgs &a, hipEvent_t ev_k0, hipEvent_t ev_k1, hipStream_t stream);
hipError_t launch_sym_finish(const SymArgs &a, const OptArgs *opt, hipStream_t stream);
// kind 2: k_phi_rows with 8-wave work-groups and the mask-free 8192-entry exp table
bool phi_rows_t8k_supported(int d, int R);
int phi_rows_t8k_rows(int R); // rows per work-group of kind 2
// full-matrix kernel scale: M = factor * sym(src) = L diag(sgn) L^T (Cholesky,
// or an eigendecomposition when M is indefinite and d <= ROWS_MAX_D);
// err = 0 positive definite, 2 indefinite, 1 non-finite / no convergence.
// wv = 2 M xc replaces 2 a xc in the phi epilogue.  work: 2 d^2 doubles.
hipError_t launch_scale_factor(const double *src, double factor, int d, double *M, double *L,
                               double *sgn, double *work, double *scal, int *err, hipStream_t stream);
hipError_t launch_prep_rec_mat(const double *xc, const double *G, const double *M, const double *L,
                               const double *sgn, int64_t n, int64_t np, int d, int KP, int RS,
                               double *rec, double *wv, hipStream_t stream);
hipError_t launch_prep_v_mat(const double *xc, const double *G, const double *M, const double *L,
                             int64_t n, int64_t np, int d, int KP, int VW, double *zc, double *V,
                             double *cvec, double *wv, hipStream_t stream);
// mode 0 (collect) needs nmax_bits from launch_mean_center (classification margin).
hipError_t launch_pair_rows(int d, int KP, int mode, int grid, const double *xc, const double *nrm,
                            const float *xf, const unsigned long long *nmax_bits,
                            int64_t n, int64_t nb, int64_t t0, int64_t t1, uint64_t *regions,
                            int64_t cap, uint32_t *counts, unsigned long long *below,
                            const SelState *st, unsigned long long *ghist, uint32_t *bpart,
                            double *dbg_out, hipStream_t stream);
// Bracket collect (mode 0 of launch_pair_rows) with fp32 MFMA classification and
// exact fp64 keys for the undecided band (d <= 16); same plan, outputs and keys.
hipError_t launch_pair_mcol(int d, int grid, const double *xc, const float *xf,
                            const unsigned long long *nmax_bits, int64_t n, int64_t nb, int64_t t0,
                            int64_t t1, uint64_t *regions, int64_t cap, uint32_t *counts,
                            unsigned long long *below, const SelState *st, uint32_t *bpart,
                            const uint32_t *xsplit, hipStream_t stream);
// (xsplit, d <= 8: the centring's split-bf16 operands -> the bf16-split Gram;
// nullptr: the f32 Gram)
// fp32 tile-path collect (k_pair_tiles<float> MODE 0 on the matrix cores,
// same keys): one region per block; KP in {4, 8, 12, 16, 32, 64}; xk: the
// key parts at KP 32 / 64 (bf16 part-product keys), else unused
hipError_t launch_pair_tcol(int KP, int grid, const float *xc, const float *nrm, const uint32_t *xk,
                            int64_t n, int64_t nb, int64_t t0, int64_t t1, uint64_t *regions,
                            int64_t cap, uint32_t *counts, unsigned long long *below,
                            const SelState *st, uint32_t *bpart, hipStream_t stream);
// F32 tile phi, streamed (k_phi_f32s): operand-ordered fp32 copies of the
// columns (XS, VS: ntiles = ceil(n / 32) tiles of 32 particles; XS holds
// ntiles * 32 * KP floats, VS ntiles * 2 * (VW/16 + 1) * 256) made by
// launch_swz_f32 from the fp64 coordinates x (stride KP), V (stride VW) and
// cvec; rows from the row-major fp32 copy xrow (stride KP) and crow.
// KP % 16 == 0 (phi_f32s_supported); row0 % 16 == 0.
hipError_t launch_swz_f32(const double *x, int KP, const double *V, int VW, const double *cvec,
                          int64_t ntiles, float *XS, float *VS, hipStream_t stream);
bool phi_f32s_supported(int KP, int NCB);
// F32 tile phi on the bf16 matrix cores (k_phi_b3: each fp32 operand as three
// bf16 parts, six part products per fp32 product): per 32-column tile
// phi_b3_tile_words(KP, NCB) dwords of operand-ordered parts made by
// launch_swz_b3 from x (stride KP), V (stride VW = 16 NCB) and cvec.
// KP = 32 or 64; row0 % 16 == 0.
bool phi_b3_supported(int KP, int NCB);
int64_t phi_b3_tile_words(int KP, int NCB);
hipError_t launch_swz_b3(const double *x, int KP, const double *V, int VW, const double *cvec,
                         int64_t n, int64_t ntiles, uint32_t *B3, hipStream_t stream);
hipError_t launch_phi_b3(int KP, int NCB, const uint32_t *B3, const float *crow,
                         const double *a_ptr, int64_t row0, int64_t nrows, int64_t ntiles, int d,
                         double inv_n, const double *wv, const double *xc, int xc_stride,
                         double *phi, const OptArgs *opt, int rg, hipStream_t stream);
// rows per work-group of k_phi_b3 with rg row groups of 16 per wave (1 or 2)
int phi_b3_rows_per_wg(int rg);
hipError_t launch_phi_f32s(int KP, int NCB, const float *XS, const float *VS, const float *xrow,
                           const float *crow, const double *a_ptr, int64_t row0, int64_t nrows,
                           int64_t ntiles, int d, double inv_n, const double *wv, const double *xc,
                           int xc_stride, double *phi, const OptArgs *opt, hipStream_t stream);
int phi_rows_blocks_per_cu(int d, int R, int kind = 0);
// G = grad log p of the Gaussian-sum model for `rows` particle rows (d <= 64)
hipError_t launch_gauss_grad(const double *X, int64_t rows, int d, int k, const double *mu,
                             const double *prec, double *G, hipStream_t stream);
hipError_t launch_finalize(const SelState *st, int navg, int src_lo, int src_hi, double logn,
                           double *a_out, double *med_out, hipStream_t stream);

} // namespace svgd_amd
