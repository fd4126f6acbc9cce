/*
 * svgd_capi.h -- C-ABI boundary of the MI355X-native SVGD inner step.
 *
 * This is the drop-in boundary for the reference's hot path
 * (khaiyichin/SVGDCpp, paths relative to the reference root):
 *
 *   SVGD::Step            include/SVGDCpp/SVGD.hpp:373-400   -> svgd_step / svgd_begin_step+svgd_finish_step
 *   SVGD::ComputePhi      include/SVGDCpp/SVGD.hpp:407-454   -> svgd_phi
 *   GaussianRBFKernel::Step/ComputeScale/ComputeMedian
 *                         include/SVGDCpp/Kernel/GaussianRBFKernel.hpp:141-156,164-188,222-254
 *                                                            -> svgd_median_scale
 *   Kernel::EvaluateKernel/EvaluateKernelGrad (RBF lambda :75-81)
 *                         include/SVGDCpp/Kernel/Kernel.hpp:279-297 -> fused inside svgd_phi
 *   Optimizer::Initialize/Step  Adam.hpp:61-83, AdaGrad.hpp:49-65, RMSProp.hpp:58-74
 *                                                            -> svgd_set_optimizer / svgd_reset_optimizer
 *   bounds setup/clamp    include/SVGDCpp/SVGD.hpp:184-216,396-399 -> svgd_set_bounds
 *   coordinate matrix     std::shared_ptr<Eigen::MatrixXd> (SVGD.hpp:494) -> svgd_set_particles / svgd_get_particles
 *
 * Conventions
 *  - Plain C types only.  Host buffers are caller-owned and only touched
 *    during the call.  Particle matrices use the reference's layout: a
 *    d x n column-major Eigen matrix, i.e. particle i occupies
 *    X[i*d .. i*d+d-1] (doubles).
 *  - A context owns all device memory and one HIP stream; it is driven by a
 *    single host thread.
 *  - Multi-GPU: one process (context) per GPU.  Particles are sharded by
 *    contiguous rows (svgd_shard); per step the context all-gathers the
 *    coordinates and log-gradients over RCCL and all-reduces the median
 *    counts.  Every rank must make the same sequence of calls.
 *  - Errors: every int-returning function returns SVGD_OK (0) or a negative
 *    SVGD_ERR_* code; svgd_last_error() gives the message, already prefixed
 *    "SVGDCpp: " like the reference's exceptions (Exceptions.hpp:16-56).
 */
#ifndef SVGDCPP_AMD_SVGD_CAPI_H
#define SVGDCPP_AMD_SVGD_CAPI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ----- return codes (mapped onto the reference's exception types by the
 *       C++ shim include/SVGDCpp/SVGD.hpp) ------------------------------ */
#define SVGD_OK 0
#define SVGD_ERR_DIM -1     /* DimensionMismatchException (SVGD.hpp:172,195,207) */
#define SVGD_ERR_UNSET -2   /* UnsetException (GaussianRBFKernel.hpp:57) */
#define SVGD_ERR_ARG -3     /* std::invalid_argument (SVGD.hpp:225-235, Adam.hpp:47) */
#define SVGD_ERR_HIP -4     /* HIP runtime failure -> std::runtime_error */
#define SVGD_ERR_RCCL -5    /* RCCL failure        -> std::runtime_error */
#define SVGD_ERR_RUNTIME -6 /* other runtime error -> std::runtime_error */

/* compute dtype of the device path (host I/O is always double).  F32 runs the
 * O(N^2) work -- median distances, kernel values, phi contraction -- on the
 * fp32 MFMA tile kernels (v_mfma_f32_16x16x4f32, v_exp_f32) for every d; the
 * O(N d) work (centring, phi epilogue, optimizer, clamp) stays fp64.  The
 * median is the exact order statistic of the fp32 distances. */
#define SVGD_F64 0
#define SVGD_F32 1

/* optimizer kinds (Optimizer/Adam.hpp, AdaGrad.hpp, RMSProp.hpp) */
#define SVGD_OPT_ADAM 0
#define SVGD_OPT_ADAGRAD 1
#define SVGD_OPT_RMSPROP 2

/* kernel scale methods (GaussianRBFKernel::ScaleMethod, GaussianRBFKernel.hpp:25-30).
 * SVGD_SCALE_FIXED is an extension: M = a*I with a user-set a (the
 * reference's "TODO: constant scale"; used by the test_svgd scenario). */
#define SVGD_SCALE_MEDIAN 0
#define SVGD_SCALE_HESSIAN 1 /* M = sum_i -hess log p(x_i) / (2 d N), GaussianRBFKernel.hpp:189-210 */
#define SVGD_SCALE_FIXED 2
#define SVGD_SCALE_MATRIX 3  /* extension: a fixed full (SPD) scale matrix M */

/* median path taken by the last svgd_median_scale / step (diagnostics) */
#define SVGD_MEDIAN_DIRECT 0   /* all pair keys stored and selected exactly */
#define SVGD_MEDIAN_BRACKET 1  /* sampled bracket + candidate selection (exact) */
#define SVGD_MEDIAN_FALLBACK 2 /* bracket missed: streamed radix select (exact) */
#define SVGD_MEDIAN_REBRACKET 3 /* bracket missed: wider bracket, collect again (exact) */

typedef struct svgd_ctx svgd_ctx;

/* ---- lifetime ---------------------------------------------------------- */

/* Single-GPU context for `dim`-dimensional particles, n of them, on HIP
 * device `device`.  Replaces SVGD's constructor allocations (SVGD.hpp:151-250). */
int svgd_create(svgd_ctx **out, int dim, int64_t n, int dtype, int device);

/* Multi-GPU context: rank `rank` of `world`, all ranks passing the same
 * 128-byte RCCL unique id (from svgd_get_unique_id on one rank, broadcast by
 * the caller by any means). */
int svgd_create_dist(svgd_ctx **out, int dim, int64_t n, int dtype, int device,
                     int world, int rank, const void *unique_id128);
int svgd_get_unique_id(void *unique_id128);
/* Measurement only (not a drop-in call): a one-GPU context that runs rank 0's
 * share of a `sim_world`-rank step -- its rows of phi and the update, its
 * share of the median's pair tiles (order statistics re-anchored inside its
 * own candidates), the host gradient on the threads one rank of sim_world
 * would get -- with no collectives, to time the per-rank work of a P-GPU run
 * on one GPU.  Its results are not the step's: svgd_get_particles,
 * svgd_get_shard, svgd_median_scale and svgd_phi return SVGD_ERR_RUNTIME, and
 * svgd_get_diagnostics reports SIM_WORLD. */
int svgd_create_sim(svgd_ctx **out, int dim, int64_t n, int dtype, int device, int sim_world);
int svgd_destroy(svgd_ctx *ctx);
const char *svgd_last_error(const svgd_ctx *ctx);

/* Rows [*row0, *row1) of the particle matrix owned by this context. */
int svgd_shard(const svgd_ctx *ctx, int64_t *row0, int64_t *row1);

/* ---- plugins ------------------------------------------------------------ */

/* Adam(lr, beta1, beta2, eps) | AdaGrad(lr, eps) | RMSProp(lr, beta=beta1, eps).
 * Argument checks and messages follow Adam.hpp:45-48, RMSProp.hpp:42-45. */
int svgd_set_optimizer(svgd_ctx *ctx, int kind, double lr, double beta1, double beta2,
                       double eps);
/* Optimizer::Initialize (zero moments, counter = 0). */
int svgd_reset_optimizer(svgd_ctx *ctx);
/* d-vector bounds; both NULL = unbounded (SVGD.hpp:184-190). */
int svgd_set_bounds(svgd_ctx *ctx, const double *lower_d, const double *upper_d);
/* SVGD_SCALE_MEDIAN (default) or SVGD_SCALE_FIXED with M = fixed_a * I. */
int svgd_set_scale(svgd_ctx *ctx, int method, double fixed_a);

/* Full-matrix kernel scale k(x, x') = exp(-(x-x')^T M (x-x')) (the
 * reference's M = kernel_parameters_[0], GaussianRBFKernel.hpp:75-81):
 *  - svgd_set_scale_matrix: a fixed symmetric positive-definite M (d x d,
 *    row-major); selects SVGD_SCALE_MATRIX.
 *  - SVGD_SCALE_HESSIAN (svgd_set_scale): every step, between
 *    svgd_begin_step and svgd_finish_step, the caller passes
 *    sum_{i in its shard} -hess log p(x_i) (d x d); the context sums it over
 *    ranks and uses M = sum / (2 d N) for that step (:189-210).
 *  The phi kernels run on z = L^T x (M = L L^T) with V_j = G_j - 2 M x_j.
 *  svgd_get_scale_matrix returns the M of the last step (a I for the
 *  isotropic methods); SVGD_ERR_RUNTIME if M was not positive definite. */
int svgd_set_scale_matrix(svgd_ctx *ctx, const double *M);
int svgd_set_step_hessian_sum(svgd_ctx *ctx, const double *H_shard_sum);
int svgd_get_scale_matrix(svgd_ctx *ctx, double *M_out);

/* ---- particles ---------------------------------------------------------- */

/* Full n x d matrix (every rank passes the full matrix). */
int svgd_set_particles(svgd_ctx *ctx, const double *X);
/* Full n x d matrix (collective in multi-GPU mode). */
int svgd_get_particles(svgd_ctx *ctx, double *X);
/* This rank's rows only ((row1-row0) x d). */
int svgd_get_shard(svgd_ctx *ctx, double *X_shard);

/* ---- the hot path ------------------------------------------------------- */

/* a = ln(n)/med^2 of the current particles (GaussianRBFKernel.hpp:168-188).
 * Either output may be NULL.  Collective in multi-GPU mode. */
int svgd_median_scale(svgd_ctx *ctx, double *a_out, double *med_out);

/* phi_hat for this rank's rows given this rank's rows of G = grad log p and
 * the scale a (SVGD.hpp:407-454).  phi_shard_out may be NULL (device only). */
int svgd_phi(svgd_ctx *ctx, const double *G_shard, double a, double *phi_shard_out);

/* One SVGD::Step (SVGD.hpp:373-400): scale from X_t, phi_hat from G_shard
 * (= grad log p at this rank's rows of X_t), optimizer increment, clamp.
 * X stays device-resident. */
int svgd_step(svgd_ctx *ctx, const double *G_shard);

/* Split step for overlapping the host log-gradient with the device median:
 * begin launches the scale computation and copies this rank's rows of X_t
 * into X_shard_out (returns once that copy is done; may be NULL); the caller
 * evaluates G there and passes it to finish. */
int svgd_begin_step(svgd_ctx *ctx, double *X_shard_out);
int svgd_finish_step(svgd_ctx *ctx, const double *G_shard);

/* Context-owned page-locked host buffers of (row1-row0) x d doubles.
 * Passing them to svgd_begin_step / svgd_finish_step avoids a staging copy. */
int svgd_host_buffers(svgd_ctx *ctx, double **x_shard, double **g_shard);

/* Block until all work queued by the context is complete. */
int svgd_sync(svgd_ctx *ctx);

/* ---- diagnostics / measurement ----------------------------------------- */

/* Scale a and median of the last step (host copies). */
int svgd_last_scale(const svgd_ctx *ctx, double *a_out, double *med_out, int *median_path);
/* The two upper-list order statistics (squared distances) the last median
 * averaged, and their ranks among the n(n-1)/2 upper-triangle distances
 * (svgd_plan_median_ranks; rank -1 = a diagonal zero, value 0).  For
 * size-independent rank checks of the selection at full size. */
int svgd_last_median_keys(svgd_ctx *ctx, double *sq_lo, double *sq_hi, int64_t *rank_lo,
                          int64_t *rank_hi);
/* HIP-event timing on the context stream.  level 1: the phi phase (median
 * end -> record prep .. reduce + update) and the median phase (previous phi
 * end -> scale final), with events only at phase boundaries; get returns the
 * accumulated milliseconds and the phi-phase count (and resets them).
 * level 2 adds the diagnostic events read by svgd_get_diagnostics -- the phi
 * kernel alone, the device's wait between the median's end and the phi chain,
 * every collective -- each one a ~5 us dispatch gap (a diagnostic pass, not
 * the timed one).  0 disables. */
int svgd_set_timing(svgd_ctx *ctx, int level);
int svgd_get_timing(svgd_ctx *ctx, double *phi_ms, double *median_ms, int64_t *count);
/* Accumulated diagnostics since the last call (then reset); writes
 * min(cap, SVGD_DIAG_LEN) doubles, returns that count or an error:
 *   STEPS            svgd_step_host_model calls
 *   PHI_KERNEL_MS/N  phi kernel alone (k_phi_rows without its reduce, or the
 *                    tile kernel), HIP events (level 2)
 *   PHI_WAIT_MS/N    device idle between the median's end and the phi chain:
 *                    waiting for the host gradient / G copies / G all-gather (level 2)
 *   COLL_MS/N        collectives on the compute stream (level 2, P > 1)
 *   GATHER_G_MS/N    the G all-gather on its own stream (level 2, P > 1)
 *   HOST_GRAD_MS     host grad log p wall time (worker thread, all chunks)
 *   HOST_XWAIT_MS    worker waiting for X_t chunk copies
 *   HOST_JOB_MS      worker job: post -> last G chunk landed
 *   HOST_WAIT_MS     calling thread waiting for the worker after queuing the median
 *   RANKS            ranks in the communicator (1 without one)
 *   HOST_THREADS     OpenMP threads of the host gradient
 *   TRK_STEPS        speculative steps whose median bracket was predicted from
 *                    the previous steps' medians (no sample, no bracket passes)
 *   TRK_MISS         of those, steps redone because the bracket missed
 *   SIM_WORLD        simulated world of a measurement context (svgd_create_sim), else 1
 *   CPU_QUOTA        CPUs of the cgroup quota (0: none); a rank's gradient
 *                    threads are at most CPU_QUOTA / world (or / SIM_WORLD)
 *   SPLIT_STEPS      steps whose phi + update ran in two row parts (the first
 *                    part's X_{t+1} feeding the next host gradient early)
 *   MIRROR_STEPS     host-model steps whose gradient read X_t from the
 *                    update's pinned mirror instead of a copy
 *   SPEC_STEPS       steps whose median took the speculative device plan
 *   G_COMM           1 if the G all-gather has its own communicator and stream */
#define SVGD_DIAG_STEPS 0
#define SVGD_DIAG_PHI_KERNEL_MS 1
#define SVGD_DIAG_PHI_KERNEL_N 2
#define SVGD_DIAG_PHI_WAIT_MS 3
#define SVGD_DIAG_PHI_WAIT_N 4
#define SVGD_DIAG_COLL_MS 5
#define SVGD_DIAG_COLL_N 6
#define SVGD_DIAG_GATHER_G_MS 7
#define SVGD_DIAG_GATHER_G_N 8
#define SVGD_DIAG_HOST_GRAD_MS 9
#define SVGD_DIAG_HOST_XWAIT_MS 10
#define SVGD_DIAG_HOST_JOB_MS 11
#define SVGD_DIAG_HOST_WAIT_MS 12
#define SVGD_DIAG_RANKS 13
#define SVGD_DIAG_HOST_THREADS 14
#define SVGD_DIAG_TRK_STEPS 15
#define SVGD_DIAG_TRK_MISS 16
#define SVGD_DIAG_SIM_WORLD 17
#define SVGD_DIAG_CPU_QUOTA 18
#define SVGD_DIAG_SPLIT_STEPS 19
#define SVGD_DIAG_MIRROR_STEPS 20
#define SVGD_DIAG_SPEC_STEPS 21
#define SVGD_DIAG_G_COMM 22
#define SVGD_DIAG_TRK_BAND 23 /* sum over tracked steps of the predicted bracket's share of the pairs */
#define SVGD_DIAG_LEN 24
int svgd_get_diagnostics(svgd_ctx *ctx, double *out, int cap);
/* Name and template arguments of the phi kernel this context launches, as
 * rocprofv3 prints them (e.g. "k_phi_rows<8, 4, 8, 8192, 8>"): the key under
 * which committed PMC profiles of that kernel are matched (bench.py). */
int svgd_phi_kernel_name(const svgd_ctx *ctx, char *buf, int cap);
/* Median tuning knobs (tests force each path): pair count at or below which
 * all keys are stored (direct path), sample size, candidate capacity.
 * Values <= 0 keep the current setting. */
int svgd_set_median_tuning(svgd_ctx *ctx, int64_t direct_max_pairs, int64_t sample_size,
                           int64_t candidate_capacity);
/* Upper-triangle squared-distance keys exactly as the device median sees
 * them, in (i<j) row-major order; n(n-1)/2 doubles (small n only). */
int svgd_debug_pair_keys(svgd_ctx *ctx, double *out, int64_t capacity);

/* ---- host-side built-in models (no GPU needed) ---------------------------
 * The target density's log-gradient stays on the host, as in the reference
 * (Model::EvaluateLogModelGrad, include/SVGDCpp/Model/Model.hpp:335-338).
 * A model here is the sum of `ncomp` unnormalised Gaussians
 * exp(-1/2 (x-mu_c)^T cov_c^-1 (x-mu_c)): ncomp = 1 is MultivariateNormal
 * (MultivariateNormal.hpp:56-61), ncomp > 1 the reference's operator+
 * composition (Model.hpp:55-92).  mus: ncomp x dim, covs: ncomp x dim x dim. */
int svgd_model_create(void **model, int dim, int ncomp, const double *mus, const double *covs);
int svgd_model_destroy(void *model);
/* G[i] = grad log p(X[i]) for nrows particles (OpenMP over rows). */
int svgd_model_logp_grad(void *model, const double *X, int64_t nrows, double *G);
/* H = sum_i -hess log p(x_i) over nrows particles (d x d, row-major): the sum
 * of the Hessian scale (GaussianRBFKernel.hpp:197-205, Model.hpp:366-370). */
int svgd_model_neg_hess_sum(void *model, const double *X, int64_t nrows, double *H);

/* One SVGD::Step (SVGD.hpp:373-400) with grad log p from a host model
 * (svgd_model_create; Model::EvaluateLogModelGrad, Model.hpp:335-338,
 * evaluated per particle as SVGD.hpp:412-416 does): svgd_begin_step +
 * svgd_model_logp_grad + svgd_finish_step with the X_t copy, the host
 * gradient and the G upload pipelined in row chunks (chunk i's gradient
 * overlaps chunk i+1's copy down and chunk i-1's copy up), so the whole host
 * round trip hides behind the device median.  Same result as the split
 * calls.  Not for SVGD_SCALE_HESSIAN (that step also needs the caller's
 * Hessian sum).  On a shard of <= 1 MiB the previous update's epilogue
 * leaves X_t in a context-private pinned buffer instead of a copy
 * (SVGD_X_MIRROR=0 disables it): the buffers of svgd_host_buffers are then
 * not guaranteed to hold X_t afterwards. */
int svgd_step_host_model(svgd_ctx *ctx, const void *model);

/* Mirror a built-in Gaussian-sum model (svgd_model_create) on the device
 * (MultivariateNormal.hpp:56-61, Model.hpp:55-92):
 * afterwards svgd_step(ctx, NULL) evaluates grad log p on the device and the
 * whole step stays in HBM.  NULL removes it.  d <= 64. */
int svgd_set_device_model(svgd_ctx *ctx, const void *model);
/* grad log p of the device model at the current particles, this rank's rows
 * (shard layout like svgd_get_shard). */
int svgd_device_logp_grad(svgd_ctx *ctx, double *G_shard_out);

/* ---- host-only planning helpers (no GPU needed) ------------------------ */

/* Row shard of rank r among `world` for n particles: equal chunks of
 * ceil(n/world) rows (trailing ranks may be short or empty). */
void svgd_plan_rows(int64_t n, int world, int rank, int64_t *row0, int64_t *row1);
/* Full-list ranks of the median (GaussianRBFKernel.hpp:222-254 over the n^2
 * distance list incl. n diagonal zeros) mapped onto the ascending list of
 * the n(n-1)/2 upper-triangle distances.  Writes up to two upper-list ranks
 * (-1 = a diagonal zero) and returns how many order statistics are averaged
 * (2 for even n^2, 1 for odd). */
int svgd_plan_median_ranks(int64_t n, int64_t *rank_lo, int64_t *rank_hi);
/* Number of block-level tiles of the median pair sweep owned by rank r
 * (row blocks of `block` particles; each unordered pair of particles is
 * visited by exactly one rank), and the (row block, column block) of tile t
 * of that rank.  The device uses block = SVGD_PAIR_BLOCK(dim) for F64 and
 * SVGD_PAIR_BLOCK_DT(dim, dtype) in general (F32: always the 64 tile). */
#define SVGD_PAIR_BLOCK(dim) ((dim) <= 16 ? 256 : 64)
#define SVGD_PAIR_BLOCK_DT(dim, dtype) ((dtype) == SVGD_F32 ? 64 : SVGD_PAIR_BLOCK(dim))
int64_t svgd_plan_pair_tiles(int64_t n, int block, int world, int rank);
void svgd_plan_pair_tile(int64_t n, int block, int world, int rank, int64_t t,
                         int64_t *row_block, int64_t *col_block);
/* Symmetric phi pass units: the (tile, sub-tile) pairs of the tile plan
 * above (blocks of `block` rows, `nsub` sub-tiles of block / nsub columns
 * per tile) in order, without the last column block's sub-tiles that hold
 * padding columns only.  svgd_plan_sym_total: their number;
 * svgd_plan_sym_unit: tile and sub-tile of unit u (returns -1 past the end). */
int64_t svgd_plan_sym_total(int64_t n, int block, int nsub);
int svgd_plan_sym_unit(int64_t n, int block, int nsub, int64_t u, int64_t *tile, int64_t *q);
/* Symmetric phi pass (k_phi_sym) plan of rank r among `world`: its
 * units [*u0, *u1) (equal pair counts per rank),
 * run by `grid` work-groups in contiguous runs; per row block P (of
 * nb = ceil(n/block)) blkg[2P] .. blkg[2P+1] = the work-groups visiting it
 * (blkg[2P+1] < blkg[2P]: none) and rbase[P] = its first row-sum record;
 * *Ia .. *Ib = the row blocks the rank's units span.  blkg holds 2 nb ints,
 * rbase nb.  Returns the number of row-sum records.  (The pass replaces the
 * reference's ComputePhi, SVGD.hpp:407-454, for d <= 8.) */
int64_t svgd_plan_sym_units(int64_t n, int block, int nsub, int world, int rank, int grid,
                            int64_t *u0, int64_t *u1, int *blkg, int *rbase, int64_t *Ia, int64_t *Ib);
/* The sharded symmetric pass's exchange (replaces the parallel branch of
 * SVGD.hpp:410-432): the rows [*r0, *r1) of rank dst's shard (svgd_plan_rows)
 * that rank src's units can add to -- the row blocks its units span and the
 * column blocks they pair with (at most (nb - 1) / 2 + 1 ahead, cyclic),
 * intersected with dst's rows (the hull of at most two pieces; *r0 == *r1:
 * none).  src sends exactly this range of its per-particle sums to dst, dst
 * receives it from src; the two sides compute the same range.  src == dst:
 * the rank's own rows it contributes to. */
void svgd_plan_sym_exchange(int64_t n, int block, int nsub, int world, int src, int dst, int64_t *r0,
                            int64_t *r1);
/* Median bucket select: from the all-reduced histogram of candidate keys in
 * `nb` ascending key-range buckets, the bucket holding each of the `nsel`
 * (1 or 2) candidate ranks, the rank inside it, and the total count of the
 * distinct selected buckets (the keys a rank compacts and all-gathers).
 * Returns 0, or -1 if a rank lies past the counted candidates. */
int svgd_plan_bucket_select(const unsigned long long *counts, int nb, int nsel,
                            const int64_t *ranks, int *bsel, int64_t *rank_in, int64_t *total);

#ifdef __cplusplus
}
#endif

#endif /* SVGDCPP_AMD_SVGD_CAPI_H */
