// svgd_capi.cpp -- C-ABI implementation: context, buffers, step orchestration.
//
// One context = one GPU (one process per GPU in multi-GPU runs).  The step
// follows SVGD::Step (reference include/SVGDCpp/SVGD.hpp:373-400):
//   kernel->Step()  -> median scale (GaussianRBFKernel.hpp:141-188)
//   ComputePhi()    -> phi_hat      (SVGD.hpp:407-454)
//   X += opt.Step() -> optimizer + clamp (SVGD.hpp:393-399)
// with X device-resident and only G (host model gradients, Model.hpp:335)
// crossing PCIe each step.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <omp.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>

#include "../../include/svgdcpp_amd/svgd_capi.h"
#include "svgd_kernels.h"
#include "hostcomm.h"
#include "host_models.h"

using namespace svgd_amd;

namespace {

constexpr int64_t TB = 64;
constexpr int XCH = 8; // row chunks of the pipelined host-gradient step
constexpr int64_t TBJ_COLS = 32; // column tile of k_phi_f32s (TBJ in svgd_kernels.hip)

struct EvPair {
    hipEvent_t a, b;
    hipEvent_t spare = nullptr; // a's own event when a is a shared mark (back to the pool)
};

// One persistent host thread per context that runs the host-gradient half of
// svgd_step_host_model (X_t chunks down -> grad log p -> G chunks up) while
// the calling thread enqueues the step's median chain: the ~14 launches
// (~5 us each) no longer sit in front of the gradient on one thread.  The
// worker spins ~1 ms after a job (the next step usually follows within it),
// then sleeps on the condition variable.
class HostWorker {
  public:
    ~HostWorker()
    {
        if (!th_.joinable()) return;
        {
            std::lock_guard<std::mutex> g(mu_);
            quit_ = true;
        }
        cv_.notify_one();
        th_.join();
    }
    void post(std::function<int(std::string &)> job)
    {
        if (!th_.joinable()) th_ = std::thread([this] { loop(); });
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = std::move(job);
            state_.store(1, std::memory_order_release);
        }
        cv_.notify_one();
    }
    // wait for the posted job; its return code (and message in err on failure)
    int wait(std::string &err)
    {
        for (int spin = 0; state_.load(std::memory_order_acquire) != 2; ++spin)
            if (spin > 64) std::this_thread::yield();
        state_.store(0, std::memory_order_relaxed);
        if (rc_) err = msg_;
        return rc_;
    }

  private:
    void loop()
    {
        for (;;) {
            const auto t0 = std::chrono::steady_clock::now();
            while (state_.load(std::memory_order_acquire) != 1 &&
                   std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(1))
                std::this_thread::yield();
            std::function<int(std::string &)> job;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [this] { return quit_ || state_.load() == 1; });
                if (quit_) return;
                job = std::move(job_);
            }
            msg_.clear();
            rc_ = job(msg_);
            state_.store(2, std::memory_order_release);
        }
    }
    std::thread th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::function<int(std::string &)> job_;
    std::atomic<int> state_{0}; // 0 idle, 1 posted, 2 done
    int rc_ = 0;
    std::string msg_;
    bool quit_ = false;
};

} // namespace

constexpr int64_t MAX_COLLECT_BLOCKS = 2048; // collect-pass grid limit (buffer sizes)
constexpr size_t XMIRROR_MAX = size_t(1) << 20; // shard bytes for the host mirror / G host read

struct svgd_ctx {
    int dim = 0;
    int64_t n = 0;
    int dtype = SVGD_F64;
    int device = 0;
    int world = 1, rank = 0;
    // svgd_create_sim (measurement only): rank 0's share of a P-rank step on
    // one GPU; every result-returning call refuses such a context
    int sim_world = 1;
    int64_t sim_pairs = 0; // the unordered pairs in that share's tiles
    int plan_world = 1;    // ranks the rows and pair tiles are planned for (world or sim_world)
    int cpu_quota = 0;     // the cgroup's CPUs (0: no quota), shared by plan_world ranks
    ncclComm_t comm = nullptr;
    // a second communicator (ncclCommSplit of comm) for the G all-gather on
    // its own stream: it overlaps the median chain's kernels and collectives
    // (one communicator's operations would run in issue order behind them).
    // On by default for P >= 2 over RCCL since round 6 (SVGD_G_COMM=0 on
    // every rank keeps the G all-gather on comm; =1 also splits a one-rank
    // communicator, the test form); the split's outcome is agreed across
    // ranks.
    //
    // Cross-communicator issue order (the invariant both communicators rely
    // on): within a step every rank issues
    //   comm:  the counts all-reduce [+ the keys all-gather when speculative]
    //          (scale_begin, all of it before returning)
    //   gcomm: the G all-gather                   (upload_g_finish)
    //   comm:  [the keys all-gather when synchronous] + the X all-gather
    // -- the same sequence on every rank because every branch in it depends on
    // all-reduced state only.  upload_g_finish checks that scale_begin has
    // issued its comm calls (coll_phase); SVGD_DEBUG_COLL=1 also all-gathers a
    // hash of each step's collective sequence and fails on any mismatch.
    ncclComm_t gcomm = nullptr;
    int coll_phase = 0;      // 0 step not begun, 1 scale_begin's comm calls issued, 2 G gathered
    uint64_t coll_sig = 0;   // FNV hash of this step's collectives (communicator, op, count)
    bool dbg_coll = false;   // SVGD_DEBUG_COLL
    uint64_t *sig_buf = nullptr; // world u64 (the debug all-gather)
    hipStream_t gstream = nullptr;
    hipEvent_t ev_gg = nullptr;   // G all-gathered (gstream)
    bool gg_pending = false;      // phi must wait for ev_gg
    HostComm *hcomm = nullptr; // SVGD_HOSTCOMM rehearsal backend (ranks sharing one GPU)
    // device mirror of a built-in Gaussian-sum model (svgd_set_device_model)
    int dm_k = 0;
    double *dm_mu = nullptr, *dm_prec = nullptr;
    int64_t row0 = 0, row1 = 0, nrows = 0, chunk = 0;
    int KP = 0, NCB = 0, VW = 0;
    int64_t nb = 0, np = 0; // row blocks; padded rows of the work arrays
    hipStream_t stream = nullptr;

    // device buffers
    double *X = nullptr;   // world*chunk x d (first n rows are the particles)
    double *G = nullptr;   // world*chunk x d
    double *xc = nullptr;  // np x KP
    double *nrm = nullptr; // np
    double *cvec = nullptr;
    double *V = nullptr;   // np x VW
    double *phi = nullptr; // nrows x d
    double *m = nullptr, *v = nullptr;
    double *lower = nullptr, *upper = nullptr;
    double *partial = nullptr;
    int nparts = 64;
    double *scal = nullptr; // [0] a, [1] med
    // SVGD_F32: fp32 copies feeding the tile kernels
    float *xcf = nullptr, *nrmf = nullptr, *cvf = nullptr, *Vf = nullptr, *zcf = nullptr;
    float *XS = nullptr, *VS = nullptr; // operand-ordered column copies (k_phi_f32s)
    uint32_t *B3 = nullptr;             // operand-ordered bf16 parts (k_phi_b3), replaces XS / VS
    uint32_t *XK = nullptr;             // F32 median key parts, KP 32 / 64 (svgd_device.h)
    bool want_b3 = false;               // F32 phi on the bf16 matrix cores (init)
    int b3_rg = 1;                      // k_phi_b3's row groups per wave (init)

    // row-stream path (d <= ROWS_MAX_D)
    bool rowpath = false;
    int RS = 0;             // record stride 2d+2
    double *rec = nullptr;  // np x RS particle records
    double *part = nullptr; // S x ldp x (d+1) phi partials
    float *xf = nullptr;    // np x med_f32_stride(d) fp32 median records
    unsigned long long *nmax = nullptr; // max |xc|^2 (double bits)
    int S = 1;
    // phi in two row parts (svgd_step_host_model when split_rows): rows
    // [0, split_h) with S2 column splits, then [split_h, nrows) with S2b
    bool split_rows = false;      // policy (init_ctx)
    bool in_host_step = false;    // run_phi_opt called by svgd_step_host_model
    bool xhalf_ready = false;     // the last step's ev_xhalf marks its first half's X_{t+1}
    int64_t split_h = 0;
    int S2 = 0, S2b = 0;
    hipEvent_t ev_xhalf = nullptr;
    int R = 2; // rows per lane of k_phi_rows
    int phi_kind = 0; // 0 k_phi_rows (4 waves: matrix scales), 2 k_phi_rows (8 waves, column-split)
    // symmetric phi pass (k_phi_sym, one rank, d <= 8): geometry and buffers
    bool sym = false;
    int symB = 0, symSRS = 0, symNSUB = 0, sym_grid = 0;
    int64_t sym_nb = 0, sym_units = 0, sym_u0 = 0, sym_u1 = 0; // all units, this rank's [u0, u1)
    int sym_fS = 1; // the row stream's column splits when it takes the step (symok = 0)
    int64_t sym_SM = 0, sym_Ia = 0, sym_Ib = 0; // colpart slots per column block; units' row-block span
    int sym_qlast = 0; // real sub-tiles of the last column block
    double *srec = nullptr, *rowpart = nullptr, *colpart = nullptr, *tab8k = nullptr;
    double *contrib = nullptr; // P > 1: every particle's sums from this rank's units (exchanged)
    // P > 1 over a communicator: the point-to-point exchange of those sums
    // (svgd_plan_sym_exchange): per rank q the rows [xsend[2q], xsend[2q+1])
    // sent to q, the rows [xrecv[3q], xrecv[3q+1]) of this rank received from
    // q into xrecv_buf + xrecv[3q+2] rows (xtab_d: xrecv on the device)
    std::vector<int64_t> xsend, xrecv;
    int64_t xrecv_rows = 0;
    double *xrecv_buf = nullptr;
    int64_t *xtab_d = nullptr;
    int *sym_tab = nullptr;    // the symmetric pass tables (SymArgs::blkg | rbase | wst)
    int *symok = nullptr;
    int64_t ldp = 0;

    // median
    int64_t direct_max_pairs = int64_t(1) << 24;
    int64_t sample_size = 0; // 0: auto, clamp(M / 256, 2^18, 2^22) for M pairs
    double bracket_sigma = 3.0; // sample-quantile standard deviations either side
    // P > 1: every rank draws the whole (smaller, <= 2^20) bracket sample of
    // the one counter-based sequence and derives the same bracket locally --
    // no histogram all-reduces in the step (two RCCL calls cost more than
    // sampling 2^20 pairs).  (shard_sample: round 2's protocol, ranks drew
    // disjoint parts of a full-size sample and all-reduced its two radix
    // histograms; kept off -- tests/test_multirank_cpu.py pins it on CPU)
    bool shard_sample = false;
    int64_t collect_blocks = 1024; // collect-pass work-groups (4 per CU resident; 5 for the bf16-split mcol)
    bool mcol = true;              // bracket collect on the matrix cores (k_pair_mcol / _tcol)
    bool mcol_bf16 = true;         // k_pair_mcol's Gram as split bf16 (d <= 8; SVGD_MCOL_BF16=0: f32)
    uint32_t *xsplit = nullptr;    // its operands, [hi | lo] bf16 x 8 per particle (the centring writes them)
    double band_est = 1.0;         // this step's bracket: expected share of the pairs
    bool samp_shard = false;    // this step's sample is sharded
    int64_t samp_local = 0;     // sample keys held by this rank
    int64_t samp_S = 0;         // this step's sample: size and target quantiles
    double samp_qlo = 0.0, samp_qhi = 0.0;
    int64_t cand_capacity = 0; // 0 = automatic
    uint64_t *sample_keys = nullptr;
    int64_t sample_alloc = 0;
    uint64_t *regions = nullptr;
    int64_t regions_alloc = 0;
    uint64_t *cbuf = nullptr;          // compacted candidates (regions_alloc keys)
    unsigned long long *ccount = nullptr;
    uint32_t *bpart = nullptr;         // collect blocks' key-range bucket histograms (max blocks x NBK)
    uint64_t *gseg = nullptr;          // world x (CAPG + 1): compacted selected-bucket keys
    int64_t bucket_cap = CAPG;         // bucket select path if the selected buckets hold <= this
    int64_t last_tot = 0;              // the last selection's selected-bucket keys (all ranks)
    int64_t spec_cap = CAPR_MIN;       // this speculative step's segment capacity (plan_step)
    uint32_t *counts = nullptr;
    unsigned long long *below = nullptr;
    int collect_grid = 0;
    int64_t nregions = 0; // candidate regions: one per wave (row-stream) or per block (tiles)
    unsigned long long *cnt3 = nullptr;
    SelState *st = nullptr;
    unsigned long long *ghist = nullptr; // [2][RADIX] radix histograms (64-bit counts)
    int64_t own_tiles = 0, tile0 = 0; // this rank's range of the median tile plan
    int pblock = 64;                  // median tile block (SVGD_PAIR_BLOCK)
    int64_t pnb = 0;                  // median row blocks

    // per-step median plan (set in begin, consumed in finish)
    int med_path = SVGD_MEDIAN_DIRECT;
    int64_t reg_cap = 0;
    int nsel = 0;
    int64_t sel_rank[2] = {0, 0};
    int src_lo = -1, src_hi = -1, navg = 1;
    bool median_pending = false;

    // pinned host
    double *h_x = nullptr, *h_g = nullptr;
    // svgd_step_host_model on a small shard (<= XMIRROR_MAX bytes): the update
    // epilogue also stores X_{t+1} into h_xm (xmirror; xh_valid while X has not
    // changed otherwise since; a buffer of its own: h_x, the caller's, is
    // never written by the device behind its back) -- no D2H copy-engine round
    // trip and cross-queue wait on the host gradient's path
    bool xmirror = false, xh_valid = false;
    // The centring fold (row path, d <= 16): X version xver (+1 per update,
    // -1 for a redo's restore, +1 and the history cleared by
    // svgd_set_particles) is centred on the mean of version xver - 1 when its
    // column partials are at hand -- the ones that version's centring left in
    // cpart[(xver - 1) & 1] -- so the centring is one launch at any P (else
    // k_mean_partial's exact mean first).  Every rank centres the same
    // all-gathered X the same way; a repeated centring of one version (a phi
    // or scale call, a redo) finds the same partials, so it forms the same
    // centre.  nmax (max |xc|^2) has a slot per version parity: a centring
    // fills its own and zeroes the other for the next.
    int64_t xver = 0;
    double *cpart = nullptr; // 2 x cpart_stride
    int64_t cpart_stride = 0;
    int cpart_n[2] = {0, 0};
    int64_t cpart_ver[2] = {-1, -1};
    double *h_xm = nullptr, *h_xm_dev = nullptr;
    unsigned long long *h_cnt = nullptr;
    double *h_scal = nullptr;
    hipEvent_t ev_x = nullptr, ev_cnt = nullptr, ev_scal = nullptr, ev_fin = nullptr;
    // host<->device copies of the X / G shards run on their own stream so
    // they overlap the median kernels; RCCL calls stay on `stream` (one
    // communicator, one issue order on every rank)
    hipStream_t cstream = nullptr;
    hipEvent_t ev_xready = nullptr, ev_g = nullptr;
    hipEvent_t ev_xch[XCH] = {};     // X_t row chunks on the host (svgd_step_host_model)

    // optimizer
    int opt_kind = -1;
    double lr = 0, b1 = 0, b2 = 0, eps = 1e-8;
    int64_t t = 0;
    bool bounded = false;
    int scale_method = SVGD_SCALE_MEDIAN;
    double fixed_a = 1.0;
    // full-matrix scale (SVGD_SCALE_MATRIX / SVGD_SCALE_HESSIAN): device M, its
    // Cholesky factor L, the (rank-summed) Hessian sum, wv = 2 M xc, zc = L^T xc
    double *sc_src = nullptr, *sc_M = nullptr, *sc_L = nullptr, *wv = nullptr, *zc = nullptr;
    double *sc_sgn = nullptr, *sc_work = nullptr; // M = L diag(sgn) L^T; Jacobi scratch
    int *sc_err = nullptr, *h_err = nullptr;
    bool hess_ready = false; // Hessian sum supplied for the current step
    std::vector<double> h_mat;
    bool have_particles = false;

    // timing (svgd_set_timing): level 1 = phase events at the phase
    // boundaries only; level 2 adds the diagnostic events (phi kernel alone,
    // the wait for G before the phi chain, every collective) -- each one a
    // dispatch gap, so a diagnostic pass, never the timed one
    bool timing = false;
    int tlevel = 0;
    std::vector<EvPair> ev_phi, ev_med;
    std::vector<EvPair> ev_pool;
    double phi_ms = 0, med_ms = 0;
    int64_t tcount = 0;
    struct DiagEv {
        hipEvent_t a, b;
        int kind;    // DG_* below
        bool own_a;  // a came from the pool (else it is a phase event)
    };
    std::vector<DiagEv> ev_diag;
    std::vector<hipEvent_t> ev_single; // pool of the diagnostic events
    hipEvent_t med_end_ev = nullptr;    // this step's median-end phase event
    double dg_ms[4] = {0, 0, 0, 0};
    int64_t dg_cnt[4] = {0, 0, 0, 0};
    // host-side wall clocks of svgd_step_host_model (always on: steady_clock)
    double h_grad_ms = 0, h_xwait_ms = 0, h_job_ms = 0, h_wait_ms = 0;
    int64_t h_steps = 0;

    int last_path = SVGD_MEDIAN_DIRECT;
    std::string err;

    // Speculative step (device-side bucket plan, no mid-step host round trip):
    // taken when the last synchronous median found the bucket path with the
    // selected buckets under CAPR.  The plan's status is copied back and
    // checked before the next call that depends on the step; a failed plan
    // (bracket miss, overflow, big buckets) restores X, m, v, t from the
    // backups and redoes the step on the synchronous path.
    bool spec_allowed = true;  // SVGD_SPECULATE=0 disables
    bool spec_step = false;    // this step's median is speculative
    bool med_ev_done = false;  // this step's median end event is recorded
    // OpenMP threads of the host gradient inside svgd_step_host_model: half the
    // host's CPUs, leaving room for this thread and the HIP runtime's -- on a
    // box whose CPU quota equals OMP_NUM_THREADS, all of them tripped the
    // cgroup throttle in ~1 of 3 runs (+0.45 ms/step at cfg3)
    int host_threads = 0;
    std::unique_ptr<HostWorker> worker; // svgd_step_host_model's gradient thread
    bool last_fast = false;    // the last resolved median could have been speculative
    bool pending = false;      // a speculative step awaits its status
    bool scal_fresh = true;    // h_scal holds the last scale (fetch_scale)
    int *d_status = nullptr, *h_status = nullptr, *h_status_dev = nullptr; // (h_status as seen by kernels)
    hipEvent_t ev_status = nullptr;
    // Every event record between two kernels costs a ~5 us dispatch gap, so
    // the end of the median records ONE event that serves as the plan status
    // (ev_status_use), the scale-final mark (ev_fin_use), the median phase's
    // end and -- while no work was queued after it (mark) -- the phi phase's
    // start.
    hipEvent_t ev_status_use = nullptr, ev_fin_use = nullptr, mark = nullptr;
    // timing off: the speculative step's status is known from this sequence
    // number, stored by the selection into h_trk[8] (no event); 0: by event
    uint64_t status_seq = 0, seq_ctr = 0;
    // likewise at the step's end: the phi phase's end event (timing) doubles
    // as X_t-final for the copy stream (ev_xready_use) when nothing follows it
    hipEvent_t phi_end = nullptr, ev_xready_use = nullptr;
    hipEvent_t last_phi_end = nullptr; // the last phi phase's end (timing): the next median's start
    double *bak = nullptr; // [X_t | m_t | v_t] of this rank's rows for the pending step

    // Bracket tracking (speculative steps): the median of D^2 moves
    // smoothly from step to step, so the collect pass's bracket is predicted
    // from the last selected keys (quadratic extrapolation, half-width 4x the
    // largest of the last 3 prediction errors) instead of a sample and its two
    // radix passes.  The selection stays exact; a bracket that misses the order
    // statistics is a failed plan, and the step is redone with a sample.
    bool trk_allowed = true;    // SVGD_TRACK_BRACKET=0 disables
    double trk_min_w = 2e-5;    // SVGD_TRACK_MIN_WIDTH: relative half-width floor
    double trk_err_mult = 4.0;  // SVGD_TRACK_ERR_MULT: half-width / recent error (set at creation)
    uint64_t *h_trk = nullptr, *h_trk_dev = nullptr; // pinned [lo, hi, below, cand, key0, key1, err]
    double trk_m[4] = {0, 0, 0, 0}; // last selected D^2 (lower order statistic), newest first
    int trk_n = 0;
    double trk_err[3] = {0, 0, 0}; // recent relative errors of the quadratic extrapolation
    int trk_nerr = 0;
    double trk_errc[3] = {0, 0, 0}; // ... and of the cubic one (4 medians)
    int trk_nerrc = 0;
    double trk_pq = -1, trk_pc = -1; // this step's two extrapolations (< 0: none)
    double trk_dens = 0;        // candidates per unit of D^2 in the last bracket (all ranks)
    double trk_pred = -1;       // this step's predicted median D^2 (< 0: sampled bracket)
    bool trk_go = false;        // this step's bracket is the predicted one (trk_plan)
    uint64_t trk_lo = 0, trk_hi = 0;
    double trk_band = 0;        // its expected share of the pairs
    bool trk_keys = false;      // this step's k_select_small writes h_trk
    // a synchronous step's selection to add to the history (resolve_pending):
    // 1 its keys are in h_trk / h_cnt, 2 it took another path (history restarts)
    int trk_sync = 0;
    int64_t trk_steps = 0, trk_miss = 0;
    double trk_band_sum = 0;    // their predicted band shares (svgd_get_diagnostics)
    // path counters (svgd_get_diagnostics): steps whose phi ran in two row
    // parts, host-model steps whose gradient read the update's pinned mirror,
    // speculative steps
    int64_t n_split = 0, n_mirror = 0, n_spec = 0;
};

namespace {

// CPUs the cgroup (v2 cpu.max "quota period", v1 cfs files) allows this
// process, rounded down; 0 = no quota or unreadable
int cgroup_cpus()
{
    long long quota = -1, period = 0;
    if (FILE *f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        if (std::fscanf(f, "%31s %lld", q, &period) == 2 && std::strcmp(q, "max") != 0)
            quota = std::atoll(q);
        std::fclose(f);
    } else {
        if (FILE *f1 = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
            if (std::fscanf(f1, "%lld", &quota) != 1) quota = -1;
            std::fclose(f1);
        }
        if (FILE *f2 = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
            if (std::fscanf(f2, "%lld", &period) != 1) period = 0;
            std::fclose(f2);
        }
    }
    return (quota > 0 && period > 0) ? (int)(quota / period) : 0;
}

int fail(svgd_ctx *c, int code, const std::string &msg)
{
    if (c) c->err = "SVGDCpp: " + msg;
    return code;
}

#define HIPCHK(c, expr)                                                                         \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return fail((c), SVGD_ERR_HIP,                                                      \
                        std::string("[HIP Error] ") + #expr + ": " + hipGetErrorString(e_));    \
    } while (0)

#define NCCLCHK(c, expr)                                                                        \
    do {                                                                                        \
        ncclResult_t r_ = (expr);                                                               \
        if (r_ != ncclSuccess)                                                                  \
            return fail((c), SVGD_ERR_RCCL,                                                     \
                        std::string("[RCCL Error] ") + #expr + ": " + ncclGetErrorString(r_));  \
    } while (0)

#define CHK(expr)                                                                               \
    do {                                                                                        \
        int rc_ = (expr);                                                                       \
        if (rc_ != SVGD_OK) return rc_;                                                         \
    } while (0)

bool pick_tiles(int d, int *KP, int *NCB)
{
    struct {
        int maxd, kp, ncb;
    } tab[] = {{4, 4, 1},   {8, 8, 1},   {12, 12, 1}, {15, 16, 1}, {16, 16, 2},
               {31, 32, 2}, {32, 32, 3}, {63, 64, 4}, {64, 64, 5}};
    for (auto &e : tab)
        if (d <= e.maxd) {
            *KP = e.kp;
            *NCB = e.ncb;
            return true;
        }
    return false;
}

template <class T> int dalloc(svgd_ctx *c, T **p, int64_t count)
{
    if (*p) {
        (void)hipFree(*p);
        *p = nullptr;
    }
    if (count <= 0) count = 1;
    HIPCHK(c, hipMalloc((void **)p, sizeof(T) * (size_t)count));
    HIPCHK(c, hipMemsetAsync(*p, 0, sizeof(T) * (size_t)count, c->stream));
    return SVGD_OK;
}

EvPair take_pair(svgd_ctx *c)
{
    EvPair p;
    if (!c->ev_pool.empty()) {
        p = c->ev_pool.back();
        c->ev_pool.pop_back();
    } else {
        (void)hipEventCreate(&p.a);
        (void)hipEventCreate(&p.b);
    }
    return p;
}

int64_t upper_pairs(int64_t n) { return n * (n - 1) / 2; }

// diagnostic event kinds (svgd_set_timing level 2; svgd_get_diagnostics)
enum { DG_PHI_KERNEL = 0, DG_PHI_WAIT = 1, DG_COLL = 2, DG_GATHER_G = 3 };

// level-2 diagnostic span on stream s: begin records a pooled event, end its
// partner; begin returns nullptr below level 2 and end then does nothing
hipEvent_t take_ev(svgd_ctx *c)
{
    hipEvent_t e = nullptr;
    if (!c->ev_single.empty()) {
        e = c->ev_single.back();
        c->ev_single.pop_back();
    } else {
        (void)hipEventCreate(&e);
    }
    return e;
}
hipEvent_t diag_begin(svgd_ctx *c, hipStream_t s)
{
    if (c->tlevel < 2) return nullptr;
    hipEvent_t e = take_ev(c);
    (void)hipEventRecord(e, s);
    c->mark = c->phi_end = nullptr; // work (an event) queued after those marks
    return e;
}
void diag_end(svgd_ctx *c, hipStream_t s, hipEvent_t a, int kind, bool own_a = true)
{
    if (!a) return;
    hipEvent_t b = take_ev(c);
    (void)hipEventRecord(b, s);
    c->ev_diag.push_back({a, b, kind, own_a});
    c->mark = c->phi_end = nullptr;
}

// ---------------------------------------------------------- collectives --

// Every collective this rank issues goes into the step's sequence hash (the
// SVGD_DEBUG_COLL cross-rank check of the issue-order invariant, svgd_ctx).
enum { CO_GATHER_ROWS = 1, CO_REDUCE_U64 = 2, CO_GATHER_U64 = 3, CO_REDUCE_F64 = 4, CO_XCHG = 6, CO_GCOMM = 16 };
void coll_note(svgd_ctx *c, int op, size_t cnt)
{
    uint64_t h = c->coll_sig ? c->coll_sig : 0xcbf29ce484222325ull;
    for (uint64_t v : {(uint64_t)op, (uint64_t)cnt}) {
        h ^= v;
        h *= 0x100000001b3ull;
    }
    c->coll_sig = h;
}

int allgather_rows_on(svgd_ctx *c, double *buf, ncclComm_t comm, hipStream_t s, int kind)
{
    if (!c->comm && !c->hcomm) return SVGD_OK; // one rank, no communicator
    c->mark = c->phi_end = nullptr; // work queued after the median's / phi's end event
    const size_t cnt = (size_t)c->chunk * c->dim;
    coll_note(c, CO_GATHER_ROWS | (comm && comm == c->gcomm ? CO_GCOMM : 0), cnt);
    hipEvent_t d0 = diag_begin(c, s);
    if (c->hcomm) {
        if (hostcomm_allgather(c->hcomm, reinterpret_cast<char *>(buf), cnt * sizeof(double), s))
            return fail(c, SVGD_ERR_RCCL, "[RCCL Error] host all-gather failed.");
    } else {
        NCCLCHK(c, ncclAllGather(buf + (size_t)c->rank * cnt, buf, cnt, ncclDouble, comm, s));
    }
    diag_end(c, s, d0, kind);
    return SVGD_OK;
}

int allgather_rows(svgd_ctx *c, double *buf)
{
    return allgather_rows_on(c, buf, c->comm, c->stream, DG_COLL);
}

int allreduce_u64(svgd_ctx *c, unsigned long long *buf, size_t cnt)
{
    if (!c->comm && !c->hcomm) return SVGD_OK; // one rank, no communicator
    coll_note(c, CO_REDUCE_U64, cnt);
    hipEvent_t d0 = diag_begin(c, c->stream);
    if (c->hcomm) {
        if (hostcomm_allreduce_u64(c->hcomm, buf, cnt, c->stream))
            return fail(c, SVGD_ERR_RCCL, "[RCCL Error] host all-reduce failed.");
    } else {
        NCCLCHK(c, ncclAllReduce(buf, buf, cnt, ncclUint64, ncclSum, c->comm, c->stream));
    }
    diag_end(c, c->stream, d0, DG_COLL);
    return SVGD_OK;
}

int allreduce_cnt3(svgd_ctx *c)
{
    // below, candidate and overflowed-region totals and the bucket counts are
    // sums; the bracket (CNT_LO, CNT_HI) is identical on every rank and stays local
    return allreduce_u64(c, c->cnt3, 3 + NBK);
}

// In-place all-gather of `cnt` u64 per rank (rank r's part at buf + r * cnt).
int allgather_u64(svgd_ctx *c, uint64_t *buf, size_t cnt)
{
    if (!c->comm && !c->hcomm) return SVGD_OK; // one rank, no communicator
    coll_note(c, CO_GATHER_U64, cnt);
    hipEvent_t d0 = diag_begin(c, c->stream);
    if (c->hcomm) {
        if (hostcomm_allgather(c->hcomm, reinterpret_cast<char *>(buf), cnt * sizeof(uint64_t),
                               c->stream))
            return fail(c, SVGD_ERR_RCCL, "[RCCL Error] host all-gather failed.");
    } else {
        NCCLCHK(c, ncclAllGather(buf + (size_t)c->rank * cnt, buf, cnt, ncclUint64, c->comm,
                                 c->stream));
    }
    diag_end(c, c->stream, d0, DG_COLL);
    return SVGD_OK;
}

// The sharded symmetric pass's exchange (the parallel branch of
// SVGD.hpp:410-432): one group of point-to-point sends and receives -- to
// each rank the range of its rows this rank's units touched, from each rank
// the range of this rank's rows its units touched (svgd_plan_sym_exchange;
// at P = 8, cfg3: ~2.5 MB per rank to ~5 peers over their direct links,
// against 4.1 MB per GPU in 7 ring steps for a reduce-scatter of all N
// sums).  k_sym_apply adds the pieces in rank order.  The host-shm
// rehearsal backend runs the same plan, and a receiver sees only what its
// senders sent (NaN elsewhere).
int sym_exchange(svgd_ctx *c)
{
    if (!c->comm && !c->hcomm) return SVGD_OK; // one rank / simulated world: no exchange
    c->mark = c->phi_end = nullptr;
    const size_t w = (size_t)c->dim + 1;
    coll_note(c, CO_XCHG, (size_t)c->n * w); // (the pieces differ by rank; the call is the same)
    hipEvent_t d0 = diag_begin(c, c->stream);
    if (c->hcomm) {
        if (hostcomm_exchange_f64(c->hcomm, c->contrib, (size_t)c->n, w, c->xsend.data(), c->xrecv_buf,
                                  (size_t)c->xrecv_rows, c->xrecv.data(), c->row0, c->row0 + c->nrows,
                                  c->stream))
            return fail(c, SVGD_ERR_RCCL, "[RCCL Error] host point-to-point exchange failed.");
    } else {
        NCCLCHK(c, ncclGroupStart());
        for (int q = 0; q < c->world; ++q) {
            if (q == c->rank) continue;
            const int64_t a = c->xsend[2 * q], b = c->xsend[2 * q + 1];
            if (b > a) NCCLCHK(c, ncclSend(c->contrib + a * w, (size_t)(b - a) * w, ncclDouble, q, c->comm, c->stream));
            const int64_t ra = c->xrecv[3 * q], rb = c->xrecv[3 * q + 1], off = c->xrecv[3 * q + 2];
            if (rb > ra)
                NCCLCHK(c, ncclRecv(c->xrecv_buf + off * w, (size_t)(rb - ra) * w, ncclDouble, q, c->comm,
                                    c->stream));
        }
        NCCLCHK(c, ncclGroupEnd());
    }
    diag_end(c, c->stream, d0, DG_COLL);
    return SVGD_OK;
}

bool matrix_scale(const svgd_ctx *c);

int allreduce_f64(svgd_ctx *c, double *buf, size_t cnt)
{
    if (!c->comm && !c->hcomm) return SVGD_OK; // one rank, no communicator
    coll_note(c, CO_REDUCE_F64, cnt);
    if (c->hcomm) {
        if (hostcomm_allreduce_f64(c->hcomm, buf, cnt, c->stream))
            return fail(c, SVGD_ERR_RCCL, "[RCCL Error] host all-reduce failed.");
        return SVGD_OK;
    }
    NCCLCHK(c, ncclAllReduce(buf, buf, cnt, ncclDouble, ncclSum, c->comm, c->stream));
    return SVGD_OK;
}

// --------------------------------------------------------------- median --

SelState make_state(int nsel, const uint64_t *ranks, uint64_t lo_key, uint64_t hi_key,
                    int known_from = 63, uint64_t prefix = 0);

// st_init (optional): the predicted bracket's select state, written by the
// centring launch itself (no launch of its own)
// Level 2: the start of the phi-wait span (run_phi) -- a pooled event of its
// own, recorded where the median ends (the phase events go back to the pool
// in svgd_get_timing; a diagnostic span must not share one of them)
int mark_median_end(svgd_ctx *c)
{
    if (c->tlevel < 2) return SVGD_OK;
    if (c->med_end_ev) c->ev_single.push_back(c->med_end_ev); // (never consumed)
    c->med_end_ev = take_ev(c);
    HIPCHK(c, hipEventRecord(c->med_end_ev, c->stream));
    c->mark = nullptr; // work (an event) queued after the median's end
    return SVGD_OK;
}

// max |xc|^2 of the current X version (its parity slot)
unsigned long long *nmax_cur(const svgd_ctx *c) { return c->nmax ? c->nmax + (c->xver & 1) : nullptr; }

int center(svgd_ctx *c, const SelState *st_init = nullptr)
{
    // the fold (svgd_ctx::cpart): the previous version's partials as the centre
    const int64_t v = c->xver;
    const int ps = (int)((v - 1) & 1), cs = (int)(v & 1);
    const bool have = c->cpart && c->cpart_ver[ps] == v - 1;
    // F32 at KP 32 / 64: the centring writes the fp32 copies itself
    const bool fused = c->dtype == SVGD_F32 && !c->rowpath && (c->KP == 32 || c->KP == 64);
    HIPCHK(c, launch_mean_center(c->X, c->n, c->dim, c->KP, c->np, c->partial, c->nparts, c->xc, c->nrm,
                                 c->rowpath ? 1 : 0, c->xf, nmax_cur(c), c->cnt3 + 3, c->stream, c->st,
                                 st_init, have ? c->cpart + ps * c->cpart_stride : nullptr,
                                 have ? c->cpart_n[ps] : 0, c->cpart ? c->cpart + cs * c->cpart_stride : nullptr,
                                 c->nmax ? c->nmax + (1 - cs) : nullptr, fused ? c->xcf : nullptr,
                                 fused ? c->nrmf : nullptr, c->xsplit));
    if (c->cpart) {
        c->cpart_ver[cs] = v;
        c->cpart_n[cs] = center_fold_grid(c->dim, c->np);
    }
    if (c->dtype == SVGD_F32) {
        if (!fused) {
            HIPCHK(c, launch_cvt_f32(c->xc, c->np * c->KP, c->xcf, c->stream));
            HIPCHK(c, launch_cvt_nrm_f32(c->nrm, c->n, c->np, c->nrmf, c->stream));
        }
        if (c->XK) HIPCHK(c, launch_swz_keys_b3(c->xcf, c->KP, c->np, c->XK, c->stream));
    }
    return SVGD_OK;
}

// Upload a fresh select state from the host.  Bits >= known_from of every
// selected key are already known to equal those of `prefix` (64: nothing
// known; keys are < 2^63); the first digit is the RADIX_BITS below them.
SelState make_state(int nsel, const uint64_t *ranks, uint64_t lo_key, uint64_t hi_key,
                    int known_from, uint64_t prefix)
{
    SelState s{};
    s.nsel = nsel;
    s.rank[0] = ranks[0];
    s.rank[1] = nsel > 1 ? ranks[1] : 0;
    const uint64_t pm = known_from >= 64 ? 0ull : ~((1ull << known_from) - 1ull);
    s.prefix[0] = s.prefix[1] = prefix & pm;
    s.shift = known_from > RADIX_BITS ? known_from - RADIX_BITS : 0;
    s.width = known_from > RADIX_BITS ? RADIX_BITS : known_from;
    s.lo_key = lo_key;
    s.hi_key = hi_key;
    s.binv = (double)NBK / (double)(hi_key - lo_key);
    return s;
}

int upload_state_s(svgd_ctx *c, const SelState &s)
{
    HIPCHK(c, launch_set_state(s, c->st, c->stream));
    return SVGD_OK;
}

int upload_state(svgd_ctx *c, int nsel, const uint64_t *ranks, uint64_t lo_key, uint64_t hi_key,
                 int known_from = 63, uint64_t prefix = 0)
{
    HIPCHK(c, launch_set_state(make_state(nsel, ranks, lo_key, hi_key, known_from, prefix), c->st,
                               c->stream));
    return SVGD_OK;
}

// One sweep over this rank's median pair tiles (mode 0 collect, 1 radix
// histogram, 2 debug dump) on the row-stream (d <= 16) or MFMA tile kernel.
hipError_t pair_pass(svgd_ctx *c, int mode, int grid, uint64_t *regions, int64_t cap, double *dbg)
{
    // the collect pass (mode 0) also histograms its candidates in key-range buckets
    uint32_t *bp = mode == 0 ? c->bpart : nullptr;
    if (c->rowpath)
        return launch_pair_rows(c->dim, c->KP, mode, grid, c->xc, c->nrm, c->xf, nmax_cur(c), c->n,
                                c->pnb, c->tile0,
                                c->tile0 + c->own_tiles, regions, cap, c->counts, c->below, c->st,
                                c->ghist, bp, dbg, c->stream);
    if (c->dtype == SVGD_F32)
        return launch_pair_tiles_f32(c->KP, mode, grid, c->xcf, c->nrmf, c->n, c->pnb, c->tile0,
                                     c->tile0 + c->own_tiles, regions, cap, c->counts, c->below,
                                     c->st, c->ghist, bp, dbg, c->XK, c->stream);
    return launch_pair_tiles(c->KP, mode, grid, c->xc, c->nrm, c->n, c->pnb, c->tile0,
                             c->tile0 + c->own_tiles, regions, cap, c->counts, c->below, c->st,
                             c->ghist, bp, dbg, c->stream);
}

constexpr double WIDE_SIGMA = 8.0; // re-bracket after a miss
// k_pair_mcol stages ~4096 x band pairs per 16-column block and wave (512
// slots): wider brackets (tiny samples, tests) take k_pair_rows' collect
constexpr double MCOL_MAX_BAND = 0.02;

SelState sample_state(svgd_ctx *c, double sigma);
int sample_bracket(svgd_ctx *c, bool preset);
int collect_counts(svgd_ctx *c);
int median_finish_spec(svgd_ctx *c, double logn);

double key_value(uint64_t k) { return __builtin_bit_cast(double, k); }

// The next median D^2 from the last 2, 3 or 4: linear, quadratic (order 2:
// on SVGD trajectories its errors are ~5x below the linear one's) or cubic
// (order 3: through 4 points; on the bench trajectories another 2-5x below
// the quadratic one's while the median still moves fast, noisier once it
// settles -- profiles/r06_track_predictor.txt)
double trk_extrapolate(const svgd_ctx *c, int order = 2)
{
    const double *m = c->trk_m;
    double p = order >= 3 && c->trk_n >= 4 ? 4.0 * m[0] - 6.0 * m[1] + 4.0 * m[2] - m[3]
               : c->trk_n >= 3          ? 3.0 * m[0] - 3.0 * m[1] + m[2]
                                        : 2.0 * m[0] - m[1];
    return p > 0.0 ? p : m[0];
}

// A resolved selection -> the tracking history: the selected lower key, the
// error of the prediction the last steps implied, the bracket's density.
void trk_record(svgd_ctx *c, uint64_t lo_key, uint64_t hi_key, uint64_t cand)
{
    const double m = key_value(c->h_trk[4]);
    if (c->h_trk[6] || !(m > 0.0) || !std::isfinite(m)) {
        c->trk_n = 0;
        return;
    }
    // both extrapolations' errors (the ones this step's plan made, else from
    // the same history)
    if (c->trk_n >= 2) {
        const double p = c->trk_pq >= 0 ? c->trk_pq : trk_extrapolate(c, 2);
        c->trk_err[2] = c->trk_err[1];
        c->trk_err[1] = c->trk_err[0];
        c->trk_err[0] = std::fabs(m - p) / m;
        c->trk_nerr = std::min(c->trk_nerr + 1, 3);
    }
    if (c->trk_n >= 4) {
        const double p = c->trk_pc >= 0 ? c->trk_pc : trk_extrapolate(c, 3);
        c->trk_errc[2] = c->trk_errc[1];
        c->trk_errc[1] = c->trk_errc[0];
        c->trk_errc[0] = std::fabs(m - p) / m;
        c->trk_nerrc = std::min(c->trk_nerrc + 1, 3);
    }
    const double lo = key_value(lo_key);
    const double hi = hi_key >= 0x7ff0000000000000ull ? INFINITY : key_value(hi_key);
    c->trk_dens = (std::isfinite(hi) && hi > lo) ? (double)cand / (hi - lo) : 0.0;
    c->trk_m[3] = c->trk_m[2];
    c->trk_m[2] = c->trk_m[1];
    c->trk_m[1] = c->trk_m[0];
    c->trk_m[0] = m;
    c->trk_n = std::min(c->trk_n + 1, 4);
}

// The predicted bracket for this step, or false (sample it): the predicted
// band must not hold more candidates than the sampled bracket's would
// (band_samp: its expected share of the pairs).  Of the quadratic and the
// cubic extrapolation, the one whose half-width -- err_mult (cubic: twice
// that) x the largest of its last 3 relative errors -- is narrower.
bool trk_predict(svgd_ctx *c, double Mq, double band_samp, uint64_t *lo_key, uint64_t *hi_key,
                 double *band_frac)
{
    if (!c->trk_allowed || c->trk_n < 2 || !(c->trk_dens > 0.0)) return false;
    const double m1 = c->trk_m[0], m2 = c->trk_m[1];
    c->trk_pq = trk_extrapolate(c, 2);
    c->trk_pc = c->trk_n >= 4 ? trk_extrapolate(c, 3) : -1.0;
    double e = 0.0;
    if (c->trk_nerr == 0) e = std::fabs(m1 - m2) / m1; // no error seen yet: the drift itself
    for (int k = 0; k < c->trk_nerr; ++k) e = std::max(e, c->trk_err[k]);
    double wp = c->trk_err_mult * e, pred = c->trk_pq;
    if (c->trk_pc >= 0 && c->trk_nerrc == 3) {
        double ec = 0.0;
        for (int k = 0; k < 3; ++k) ec = std::max(ec, c->trk_errc[k]);
        if (2.0 * c->trk_err_mult * ec < wp) {
            wp = 2.0 * c->trk_err_mult * ec;
            pred = c->trk_pc;
        }
    }
    const double w = std::max(wp, c->trk_min_w);
    const double band = c->trk_dens * (2.0 * w * pred) / Mq;
    if (!(w < 0.05)) return false;
    const double lo = pred * (1.0 - w), hi = pred * (1.0 + w);
    if (!(band <= band_samp)) return false;
    *lo_key = __builtin_bit_cast(uint64_t, lo);
    *hi_key = __builtin_bit_cast(uint64_t, hi) + 1;
    *band_frac = band;
    c->trk_pred = pred;
    return true;
}

// The default sample size of the bracket passes for M unordered pairs.
int64_t sample_size(const svgd_ctx *c, int64_t M)
{
    // sample size: the band it leaves costs the collect pass, sampling and
    // the two bracket passes cost ~S; measured optimum near M / 256 pairs
    // (cfg2, M = 1.3e8: 2^19 -> median 0.222 vs 0.262 ms at 2^22), capped
    // at 2^22 (cfg3, M = 2.1e9)
    // tile path: whole random 64 x 64 tiles (MFMA Gram, ~1/1000 of the
    // collect pass) instead of scattered pairs (2 random 8d-byte rows each).
    // Its keys come in correlated 4096-key tiles, so it keeps 2^22 (1024
    // tiles) whatever M: the bracket's sigma assumes many independent draws.
    const bool tile_path = !c->rowpath && c->n / TB >= 2;
    int64_t S = c->sample_size > 0 ? c->sample_size
                : tile_path       ? int64_t(1) << 22
                                  : std::min<int64_t>(std::max<int64_t>(M / 256, int64_t(1) << 18),
                                                      int64_t(1) << 22);
    const bool multi = c->comm || c->hcomm || c->sim_world > 1;
    if (multi && !c->shard_sample && c->sample_size <= 0)
        S = std::min<int64_t>(S, int64_t(1) << 20); // every rank draws all of it
    return std::min<int64_t>(S, M);
}

// This step's bracket, decided before the centring launch (which then also
// writes the predicted select state): predicted on speculative steps (row
// and tile paths: keys are D^2 as doubles on both) when trk_predict allows
// it, else sampled in median_begin.
void trk_plan(svgd_ctx *c)
{
    c->trk_go = false;
    c->trk_pred = -1;
    c->trk_pq = c->trk_pc = -1;
    const int64_t M = upper_pairs(c->n);
    if (!c->spec_step || c->sample_size > 0 || c->cand_capacity > 0 || M <= c->direct_max_pairs)
        return;
    const int64_t S = sample_size(c, M);
    const double Mq = c->sim_world > 1 ? (double)c->sim_pairs : (double)M;
    // the sampled bracket's expected share (sample_state at q = 1/2; whole-tile
    // samples take 4x the sigmas, median_begin)
    const bool tile_sample = !c->rowpath && c->n / TB >= 2 && S >= TB * TB;
    const double sigma = tile_sample ? 4.0 * c->bracket_sigma : c->bracket_sigma;
    const double sig = std::sqrt((double)S * 0.25) + 1.0;
    const double band_samp = (2.0 * sigma * sig + 3.0) / (double)S;
    c->trk_go = trk_predict(c, Mq, band_samp, &c->trk_lo, &c->trk_hi, &c->trk_band);
}

// Phase 1 of the median: candidate bracket + collect pass + counts.
// Leaves the reduced counts in c->h_cnt (ready at c->ev_cnt).
int median_begin(svgd_ctx *c)
{
    c->trk_keys = false;
    const int64_t n = c->n;
    int64_t rlo, rhi;
    c->navg = svgd_plan_median_ranks(n, &rlo, &rhi);
    if (c->sim_world > 1 && rlo >= 0) { // the same quantile of this rank's share of the pairs
        const int64_t d = rhi - rlo;
        rlo = (int64_t)((long double)rlo * (long double)c->sim_pairs / (long double)upper_pairs(n));
        rhi = rlo + d;
    }
    // distinct non-negative upper ranks to select
    c->nsel = 0;
    c->src_lo = c->src_hi = -1;
    if (rlo >= 0) {
        c->sel_rank[c->nsel] = rlo;
        c->src_lo = c->nsel++;
    }
    if (rhi >= 0) {
        if (c->nsel == 1 && rhi == rlo) {
            c->src_hi = 0;
        } else {
            c->sel_rank[c->nsel] = rhi;
            c->src_hi = c->nsel++;
        }
    }
    if (c->navg == 1) c->src_hi = c->src_lo;
    c->median_pending = true;
    if (c->nsel == 0) { // med = 0 (n <= 1 or all diagonal)
        c->med_path = SVGD_MEDIAN_DIRECT;
        return SVGD_OK;
    }

    const int64_t M = upper_pairs(n);
    const int64_t tiles = c->own_tiles;
    c->collect_grid = (int)std::max<int64_t>(1, std::min<int64_t>(tiles, c->collect_blocks));
    c->nregions = c->rowpath ? 4 * (int64_t)c->collect_grid : c->collect_grid;
    const int64_t tiles_per_blk = (tiles + c->nregions - 1) / c->nregions;

    if (M <= c->direct_max_pairs) {
        // every key is a candidate: bracket [0, ~0)
        c->med_path = SVGD_MEDIAN_DIRECT;
        c->reg_cap = tiles_per_blk * c->pblock * c->pblock;
        uint64_t z[2] = {0, 0};
        CHK(upload_state(c, 1, z, 0, ~0ull));
    } else {
        c->med_path = SVGD_MEDIAN_BRACKET;
        const bool tile_path = !c->rowpath && n / TB >= 2;
        int64_t S = sample_size(c, M);
        const double Mq = c->sim_world > 1 ? (double)c->sim_pairs : (double)M;
        if (c->trk_go) {
            // predicted bracket (trk_plan; its select state was written by
            // the centring launch): no sample, no radix passes (k_center
            // zeroed the bucket counts); regions sized for 4x the band
            c->trk_steps += 1;
            c->trk_band_sum += c->trk_band;
            c->band_est = c->trk_band;
            const int64_t pairs_own = tiles * c->pblock * c->pblock;
            const int64_t total = (int64_t)(4.0 * c->trk_band * (double)pairs_own) + 2048 * c->nregions;
            c->reg_cap = std::max<int64_t>(1, total / c->nregions);
            const int64_t need = c->reg_cap * c->nregions;
            if (c->regions_alloc < need) {
                CHK(dalloc(c, &c->regions, need));
                CHK(dalloc(c, &c->cbuf, need));
                c->regions_alloc = need;
            }
            return collect_counts(c);
        }
        if (c->sim_world > 1 && c->shard_sample) S = std::max<int64_t>(1, S / c->sim_world); // a rank's share
        const bool tile_sample = tile_path && S >= TB * TB;
        if (tile_sample) S = S / (TB * TB) * (TB * TB);
        if (c->sample_alloc < S) {
            CHK(dalloc(c, &c->sample_keys, S));
            c->sample_alloc = S;
        }
        if (tile_sample)
            HIPCHK(c, launch_sample_tiles(c->KP, c->xc, c->nrm, c->xcf, c->nrmf, c->XK, n,
                                          S / (TB * TB), c->sample_keys, c->stream));
        // sharded (P > 1, scattered pairs): rank r draws pairs [S r/P, S (r+1)/P)
        // of the one counter-based sequence and the bracket's histograms are
        // all-reduced -- the same sample, hence the same bracket, as on one rank
        c->samp_shard = !tile_sample && (c->comm || c->hcomm) && c->shard_sample;
        const int64_t g0 = c->samp_shard ? S * c->rank / c->world : 0;
        c->samp_local = c->samp_shard ? S * (c->rank + 1) / c->world - g0 : S;
        c->samp_S = S;
        c->samp_qlo = (double)c->sel_rank[0] / Mq;
        c->samp_qhi = (double)c->sel_rank[c->nsel - 1] / Mq;
        // whole-tile samples are correlated (a far particle shifts its tile's
        // 64 x 64 keys together): 3 sigma of S independent draws missed the
        // bracket on ~40 % of cfg5 steps (each miss: a second collect pass);
        // 12 measured none at no cost (the band stays ~1 % of the pairs)
        const SelState init = sample_state(c, tile_sample ? 4.0 * c->bracket_sigma : c->bracket_sigma);
        if (!tile_sample)
            HIPCHK(c, launch_sample_keys(c->xc, c->nrm, c->xf, n, c->dim, c->KP, g0, c->samp_local,
                                         c->sample_keys, init, c->st, c->stream));
        else
            HIPCHK(c, launch_set_state(init, c->st, c->stream));
        CHK(sample_bracket(c, true));
        int64_t pairs_own = tiles * c->pblock * c->pblock;
        int64_t total = c->cand_capacity;
        if (total <= 0) {
            const double frac = (c->samp_qhi - c->samp_qlo) + 16.0 / std::sqrt((double)S) + 0.004;
            total = (int64_t)(2.0 * frac * (double)pairs_own) + 2048 * c->nregions;
        }
        c->reg_cap = std::max<int64_t>(1, total / c->nregions);
    }
    const int64_t need = c->reg_cap * c->nregions;
    if (c->regions_alloc < need) {
        CHK(dalloc(c, &c->regions, need));
        CHK(dalloc(c, &c->cbuf, need));
        c->regions_alloc = need;
    }
    return collect_counts(c);
}

// Sample ranks bracketing the target quantiles (sigma sample-quantile standard
// deviations either side): the select state of the bracket passes.
SelState sample_state(svgd_ctx *c, double sigma)
{
    const int64_t S = c->samp_S;
    const double qlo = c->samp_qlo, qhi = c->samp_qhi;
    const double sig_lo = std::sqrt((double)S * qlo * (1 - qlo)) + 1.0;
    const double sig_hi = std::sqrt((double)S * qhi * (1 - qhi)) + 1.0;
    double slo = std::floor(qlo * S - sigma * sig_lo) - 1;
    double shi = std::ceil(qhi * S + sigma * sig_hi) + 1;
    if (slo < 0) slo = 0;
    if (shi > S - 1) shi = (double)(S - 1);
    const uint64_t sr[2] = {(uint64_t)slo, (uint64_t)shi};
    c->band_est = (shi - slo + 1.0) / (double)S; // expected share of pairs in the bracket
    return make_state(2, sr, 0, ~0ull);
}

// The two radix passes over the sample from that state (already on the device
// if preset: the sampler wrote it) -> bracket [lo_key, hi_key), which stays on
// the device (read by the collect pass).  Per pass: one histogram launch
// (atomics into ghist), the all-reduce if the sample is sharded, one scan
// launch; the last scan also sets the bracket.
int sample_bracket(svgd_ctx *c, bool preset)
{
    (void)preset;
    for (int p = 0; p < 2; ++p) {
        HIPCHK(c, launch_hist_regions(c->sample_keys, nullptr, 1, c->samp_local, 0, c->st, c->ghist,
                                      c->stream));
        if (c->samp_shard) CHK(allreduce_u64(c, c->ghist, 2 * RADIX));
        HIPCHK(c, launch_select_scan(c->st, c->ghist, p == 1, c->cnt3 + 3, c->stream));
    }
    return SVGD_OK;
}

// Collect pass over this rank's pair tiles, then the all-reduced counts to the
// host (ready at ev_cnt).
int collect_counts(svgd_ctx *c)
{
    if (c->rowpath && c->mcol && c->med_path != SVGD_MEDIAN_DIRECT && c->band_est <= MCOL_MAX_BAND)
        // bracket collect: fp32 MFMA classification, exact keys for the band
        // (a thin band only: each band pair is staged and finished one by one)
        HIPCHK(c, launch_pair_mcol(c->dim, c->collect_grid, c->xc, c->xf, nmax_cur(c), c->n, c->pnb,
                                   c->tile0, c->tile0 + c->own_tiles, c->regions, c->reg_cap,
                                   c->counts, c->below, c->st, c->bpart, c->xsplit, c->stream));
    else if (!c->rowpath && c->dtype == SVGD_F32 && c->mcol)
        // fp32 tile path: k_pair_tiles' keys, rows held in VGPRs, no LDS
        HIPCHK(c, launch_pair_tcol(c->KP, c->collect_grid, c->xcf, c->nrmf, c->XK, c->n, c->pnb,
                                   c->tile0, c->tile0 + c->own_tiles, c->regions, c->reg_cap,
                                   c->counts, c->below, c->st, c->bpart, c->stream));
    else
        HIPCHK(c, pair_pass(c, 0, c->collect_grid, c->regions, c->reg_cap, nullptr));
    HIPCHK(c, launch_counts_reduce(c->below, c->counts, c->nregions, c->reg_cap, c->st, c->bpart,
                                   c->collect_grid, c->cnt3, c->stream,
                                   c->spec_step ? c->gseg + (size_t)c->rank * (c->spec_cap + 1) : nullptr));
    CHK(allreduce_cnt3(c));
    // speculative: the device plan and the selection are queued right behind
    // the counts (while the device still runs the collect pass), not when the
    // host comes back from the gradient -- no launch gaps between them
    if (c->spec_step) return median_finish_spec(c, std::log((double)c->n));
    HIPCHK(c, hipMemcpyAsync(c->h_cnt, c->cnt3, CNT_LEN * sizeof(unsigned long long),
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipEventRecord(c->ev_cnt, c->stream));
    return SVGD_OK;
}

// Speculative phase 2: plan, compact, gather and select on the device; the
// plan's status goes to the host on the copy stream (resolve_pending).
int median_finish_spec(svgd_ctx *c, double logn)
{
    const int64_t cap = c->spec_cap;
    uint64_t *seg = c->gseg + (size_t)c->rank * (cap + 1);
    // the plan also stores its status straight into pinned host memory: no
    // copy on the copy stream (a small copy there turned the X shard copies
    // into blit kernels competing with the median kernels)
    // (the compaction's blocks derive the bucket plan themselves: no plan launch)
    const PlanArgs pa{c->cnt3, c->nsel, (uint64_t)c->sel_rank[0], (uint64_t)c->sel_rank[c->nsel - 1],
                      cap, c->d_status, c->h_status_dev,
                      c->sim_world > 1 ? 1 : 0, c->h_trk_dev};
    HIPCHK(c, launch_compact_buckets(c->regions, c->counts, c->nregions, c->reg_cap, c->st, seg, cap,
                                     c->d_status, c->stream, &pa));
    CHK(allgather_u64(c, c->gseg, (size_t)cap + 1));
    // the plan's status is final once the selection completes.  Timing off
    // (the product path): no event at all -- the selection stores a sequence
    // number into pinned memory after its last store and resolve_pending
    // polls it (an event between two kernels costs a ~6 us dispatch gap,
    // profiles/r06_step_timeline_*); with phase timing the phase event there
    // serves.  (c->pending -- the plan's status to check -- is set when the
    // step is complete, by median_finish: resolve_pending never redoes half a
    // step.)
    const bool by_seq = !c->timing && c->tlevel < 2;
    c->status_seq = by_seq ? ++c->seq_ctr : 0;
    HIPCHK(c, launch_select_small(c->st, c->gseg, c->world, cap, c->navg, c->src_lo, c->src_hi, logn,
                                  c->scal, c->d_status, c->stream, c->h_trk_dev, c->status_seq));
    c->trk_keys = true;
    if (by_seq) {
        c->ev_status_use = nullptr;
        c->med_ev_done = true; // (no scale-final event either: fetch_scale syncs the stream)
        c->mark = nullptr;
        return SVGD_OK;
    }
    if (c->timing && !c->ev_med.empty()) {
        c->ev_status_use = c->ev_med.back().b; // also the median phase's end
        c->med_ev_done = true;
        c->mark = c->ev_status_use;
    } else {
        c->ev_status_use = c->ev_status;
    }
    HIPCHK(c, hipEventRecord(c->ev_status_use, c->stream));
    CHK(mark_median_end(c));
    return SVGD_OK;
}

// Phase 2: exact selection among candidates (or streamed fallback), then a.
int median_finish(svgd_ctx *c)
{
    if (!c->median_pending) return fail(c, SVGD_ERR_RUNTIME, "[Runtime Error] median not begun.");
    c->median_pending = false;
    const double logn = std::log((double)c->n);
    if (c->nsel == 0) {
        // every averaged order statistic is a diagonal zero
        uint64_t z[2] = {0, 0};
        CHK(upload_state(c, 1, z, 0, 0));
        HIPCHK(c, launch_finalize(c->st, c->navg, -1, -1, logn, c->scal, c->scal + 1, c->stream));
        c->last_path = SVGD_MEDIAN_DIRECT;
        return SVGD_OK;
    }
    if (c->spec_step) { // queued by collect_counts
        c->pending = true;
        c->last_path = c->med_path;
        return SVGD_OK;
    }
    c->last_fast = false;
    HIPCHK(c, hipEventSynchronize(c->ev_cnt));
    if (c->sim_world > 1 && !c->h_cnt[2] && c->h_cnt[1] > 0) {
        // measurement mode: the share is selected alone -- re-anchor the
        // ranks inside its candidates (the device plan does the same)
        const int64_t dr = c->sel_rank[c->nsel - 1] - c->sel_rank[0];
        c->sel_rank[0] = (int64_t)(c->h_cnt[0] + c->h_cnt[1] / 2);
        if (c->nsel > 1) c->sel_rank[1] = c->sel_rank[0] + dr;
    }
    const uint64_t r0 = (uint64_t)c->sel_rank[0], r1 = (uint64_t)c->sel_rank[c->nsel - 1];
    auto in_bracket = [&]() {
        return !c->h_cnt[2] && r0 >= c->h_cnt[0] && r1 < c->h_cnt[0] + c->h_cnt[1];
    };
    int path = c->med_path;
    if (!in_bracket() && path == SVGD_MEDIAN_BRACKET && !c->h_cnt[2]) {
        // the order statistics fell outside the sampled bracket (probability
        // ~2e-3 per step at the default 3 sigma): bracket again from the same
        // sample at WIDE_SIGMA and repeat the collect pass (one more pass)
        // instead of the streamed radix select (one pass per 11-bit digit)
        CHK(upload_state_s(c, sample_state(c, std::max(c->bracket_sigma, WIDE_SIGMA))));
        CHK(sample_bracket(c, false));
        CHK(collect_counts(c));
        HIPCHK(c, hipEventSynchronize(c->ev_cnt));
        path = SVGD_MEDIAN_REBRACKET;
    }
    const unsigned long long below = c->h_cnt[0];
    const uint64_t lo_key = c->h_cnt[CNT_LO], hi_key = c->h_cnt[CNT_HI];
    bool ok = in_bracket();
    uint64_t ranks[2];
    if (ok) {
        ranks[0] = c->sel_rank[0] - below;
        ranks[1] = c->sel_rank[c->nsel - 1] - below;
    } else {
        path = SVGD_MEDIAN_FALLBACK;
        ranks[0] = c->sel_rank[0];
        ranks[1] = c->sel_rank[c->nsel - 1];
    }
    // Bucket select: the collect pass histogrammed the candidates in NBK
    // key-range buckets (all-reduced with the counts), so the bucket holding
    // each order statistic is known here.  If those buckets are small, every
    // rank compacts its keys in them, the compacted keys are all-gathered once
    // and one work-group selects exactly -- no per-digit all-reduces.
    if (ok && c->bucket_cap > 0) {
        const int64_t rr[2] = {(int64_t)ranks[0], (int64_t)ranks[1]};
        int bsel[2];
        int64_t rin[2], tot = 0;
        const int ns = (c->nsel > 1 && ranks[1] != ranks[0]) ? 2 : 1;
        if (svgd_plan_bucket_select(c->h_cnt + 3, NBK, ns, rr, bsel, rin, &tot) == 0 &&
            tot <= std::min<int64_t>(c->bucket_cap, CAPG)) {
            // one segment per rank, sized for the selected buckets' total (a
            // rank holds at most that many): the all-gather moves tot keys per
            // rank, not the CAPG capacity
            const int64_t scap = std::max<int64_t>(1, tot);
            uint64_t *seg = c->gseg + (size_t)c->rank * (scap + 1);
            HIPCHK(c, launch_set_sel(c->st, c->nsel, (uint64_t)rin[0],
                                     (uint64_t)(c->nsel > 1 ? rin[ns - 1] : rin[0]), bsel[0],
                                     bsel[ns - 1], seg, c->stream));
            HIPCHK(c, launch_compact_buckets(c->regions, c->counts, c->nregions, c->reg_cap, c->st,
                                             seg, scap, nullptr, c->stream));
            CHK(allgather_u64(c, c->gseg, (size_t)scap + 1));
            HIPCHK(c, launch_select_small(c->st, c->gseg, c->world, scap, c->navg, c->src_lo,
                                          c->src_hi, logn, c->scal, nullptr, c->stream, c->h_trk_dev));
            c->trk_keys = true;
            c->last_path = path;
            // the next step may take the device plan if this one would have
            c->last_fast = (path == SVGD_MEDIAN_BRACKET || path == SVGD_MEDIAN_DIRECT) &&
                           tot <= std::min<int64_t>(c->bucket_cap, CAPG);
            c->last_tot = tot;
            return SVGD_OK;
        }
    }
    // every candidate key lies in [lo_key, hi_key): their common leading bits
    // are known, so the radix passes start below them (bracket path only)
    int known_from = 63;
    if ((path == SVGD_MEDIAN_BRACKET || path == SVGD_MEDIAN_REBRACKET) && hi_key > lo_key) {
        const uint64_t diff = lo_key ^ (hi_key - 1);
        known_from = diff ? 64 - __builtin_clzll(diff) : 0;
        if (known_from > 63) known_from = 63;
    }
    CHK(upload_state(c, c->nsel, ranks, 0, ~0ull, known_from, lo_key));
    const int passes = (known_from + RADIX_BITS - 1) / RADIX_BITS;
    if (path == SVGD_MEDIAN_FALLBACK) {
        // streamed radix select over every pair (rare: the bracket missed)
        for (int p = 0; p < passes; ++p) {
            const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(c->own_tiles, 2048));
            HIPCHK(c, pair_pass(c, 1, grid, nullptr, 0, nullptr));
            CHK(allreduce_u64(c, c->ghist, 2 * RADIX));
            HIPCHK(c, launch_select_scan(c->st, c->ghist, 0, nullptr, c->stream));
        }
    } else if (passes > 0) {
        // first digit over every candidate, then only the keys in the chosen
        // bucket(s) are kept (compacted) for the remaining digits
        HIPCHK(c, launch_hist_regions(c->regions, c->counts, c->nregions, c->reg_cap, 0, c->st,
                                      c->ghist, c->stream));
        CHK(allreduce_u64(c, c->ghist, 2 * RADIX));
        HIPCHK(c, launch_select_scan(c->st, c->ghist, 0, nullptr, c->stream));
        if (passes > 1) {
            HIPCHK(c, launch_compact(c->regions, c->counts, c->nregions, c->reg_cap, c->st, c->cbuf,
                                     c->ccount, c->stream));
            if (!c->comm && !c->hcomm) {
                // remaining digits in one work-group, no launches in between
                HIPCHK(c, launch_select_tail(c->st, c->cbuf, c->ccount, passes - 1, c->stream));
            } else {
                for (int p = 1; p < passes; ++p) {
                    HIPCHK(c, launch_hist_count(c->cbuf, c->ccount, c->regions_alloc, c->st,
                                                c->ghist, c->stream));
                    CHK(allreduce_u64(c, c->ghist, 2 * RADIX));
                    HIPCHK(c, launch_select_scan(c->st, c->ghist, 0, nullptr, c->stream));
                }
            }
        }
    }
    HIPCHK(c, launch_finalize(c->st, c->navg, c->src_lo, c->src_hi, logn, c->scal, c->scal + 1,
                              c->stream));
    c->last_path = path;
    return SVGD_OK;
}

int check_ready(svgd_ctx *c)
{
    if (!c) return SVGD_ERR_ARG;
    if (!c->have_particles)
        return fail(c, SVGD_ERR_UNSET, "[Unset Error] Particle coordinates are unset.");
    return SVGD_OK;
}

// Calls that hand results back refuse a measurement context (svgd_create_sim):
// its particles, phi and scale are one rank's share computed without the
// other ranks' data, not the step's.
int check_results(svgd_ctx *c)
{
    CHK(check_ready(c));
    if (c->sim_world > 1)
        return fail(c, SVGD_ERR_RUNTIME,
                    "[Runtime Error] measurement context (svgd_create_sim, world " +
                        std::to_string(c->sim_world) + "): its results are not the step's.");
    return SVGD_OK;
}

// G shard -> device on the copy stream (ready at ev_g) ...
int upload_g_begin(svgd_ctx *c, const double *G_shard)
{
    const size_t bytes = sizeof(double) * (size_t)c->nrows * c->dim;
    if (!G_shard) return fail(c, SVGD_ERR_ARG, "[Argument Error] Null log-gradient buffer.");
    if (c->nrows > 0) {
        if (G_shard != c->h_g) {
            HIPCHK(c, hipEventSynchronize(c->ev_g)); // the previous upload left h_g
            std::memcpy(c->h_g, G_shard, bytes);
        }
        HIPCHK(c, hipMemcpyAsync(c->G + (size_t)c->row0 * c->dim, c->h_g, bytes,
                                 hipMemcpyHostToDevice, c->cstream));
    }
    HIPCHK(c, hipEventRecord(c->ev_g, c->cstream));
    return SVGD_OK;
}

// ... and the all-gather of the shards.  With a G communicator (P > 1 over
// RCCL) it runs on its own stream as soon as the shard has landed, beside the
// median chain, and the phi chain waits for it (run_phi); otherwise on the
// compute stream once it needs G.
int upload_g_finish(svgd_ctx *c)
{
    if (c->gcomm) {
        // the issue-order invariant (svgd_ctx): with a median pending, every
        // comm call of scale_begin precedes this gcomm call on every rank
        if (c->median_pending && c->coll_phase != 1)
            return fail(c, SVGD_ERR_RUNTIME,
                        "[Runtime Error] G all-gather issued before the median's collectives "
                        "(cross-communicator issue order).");
        c->coll_phase = 2;
        if (hipEventQuery(c->ev_g) != hipSuccess) HIPCHK(c, hipStreamWaitEvent(c->gstream, c->ev_g, 0));
        CHK(allgather_rows_on(c, c->G, c->gcomm, c->gstream, DG_GATHER_G));
        HIPCHK(c, hipEventRecord(c->ev_gg, c->gstream));
        c->gg_pending = true;
        return SVGD_OK;
    }
    // a G copy that has already landed needs no cross-queue barrier (a wait
    // on the copy stream's signal cost a ~25 us dispatch gap before the
    // record prep even when the copy had finished long before)
    if (hipEventQuery(c->ev_g) != hipSuccess) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_g, 0));
    CHK(allgather_rows(c, c->G));
    return SVGD_OK;
}

int upload_g(svgd_ctx *c, const double *G_shard)
{
    CHK(upload_g_begin(c, G_shard));
    return upload_g_finish(c);
}

bool matrix_scale(const svgd_ctx *c)
{
    return c->scale_method == SVGD_SCALE_MATRIX || c->scale_method == SVGD_SCALE_HESSIAN;
}

// F32 with the streamed tile phi (operand-ordered copies allocated, 16-aligned rows)
bool phi_streamed(const svgd_ctx *c)
{
    return c->dtype == SVGD_F32 && (c->XS || c->B3) && c->row0 % 16 == 0;
}

int run_phi(svgd_ctx *c, const OptArgs *opt)
{
    // phi phase: the record preparation (V = G - 2a xc, part of the
    // reference's ComputePhi) through the reduce (+ the fused update); the
    // start event goes before the preparation -- an event between two
    // kernels costs a dispatch gap
    EvPair ev{};
    if (c->timing) {
        ev = take_pair(c);
        if (c->mark) { // the median's end event, nothing queued since
            ev.spare = ev.a;
            ev.a = c->mark;
        } else {
            HIPCHK(c, hipEventRecord(ev.a, c->stream));
        }
    }
    // level 2: the device's wait between the median's end and the phi chain
    // (the host gradient, the G copies and, P > 1, the G all-gather)
    hipEvent_t med_end = c->tlevel >= 2 ? c->med_end_ev : nullptr;
    c->med_end_ev = nullptr;
    c->mark = nullptr;
    if (c->gg_pending) {
        if (hipEventQuery(c->ev_gg) != hipSuccess) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_gg, 0));
        c->gg_pending = false;
    }
    if (med_end) diag_end(c, c->stream, med_end, DG_PHI_WAIT, true);
    const bool mat = matrix_scale(c);
    if (mat) {
        // M = factor * src, L = chol(M), a_eff = 1 (GaussianRBFKernel.hpp:189-210)
        const double factor = c->scale_method == SVGD_SCALE_HESSIAN
                                  ? 1.0 / (2.0 * (double)c->dim * (double)c->n)
                                  : 1.0;
        HIPCHK(c, launch_scale_factor(c->sc_src, factor, c->dim, c->sc_M, c->sc_L, c->sc_sgn,
                                      c->sc_work, c->scal, c->sc_err, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->h_err, c->sc_err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        if (!c->rowpath) {
            // the MFMA tile kernels need M positive definite: check before phi
            HIPCHK(c, hipStreamSynchronize(c->stream));
            if (*c->h_err == 2)
                return fail(c, SVGD_ERR_RUNTIME,
                            "[Runtime Error] The kernel scale matrix is indefinite; the device "
                            "path supports indefinite matrices for fp64 particles with d <= 16 only.");
        }
        if (*c->h_err == 1 && !c->rowpath)
            return fail(c, SVGD_ERR_RUNTIME, "[Runtime Error] The kernel scale matrix is not finite.");
        if (c->rowpath)
            HIPCHK(c, launch_prep_rec_mat(c->xc, c->G, c->sc_M, c->sc_L, c->sc_sgn, c->n, c->np,
                                          c->dim, c->KP, c->RS, c->rec, c->wv, c->stream));
        else
            HIPCHK(c, launch_prep_v_mat(c->xc, c->G, c->sc_M, c->sc_L, c->n, c->np, c->dim, c->KP,
                                        c->VW, c->zc, c->V, c->cvec, c->wv, c->stream));
    } else if (c->rowpath && !c->sym) // (the symmetric pass's prep writes these when it does not apply)
        HIPCHK(c, launch_prep_rec(c->xc, c->G, c->nrm, c->scal, c->n, c->np, c->dim, c->KP, c->RS,
                                  c->rec, c->stream));
    else if (!c->rowpath)
        HIPCHK(c, launch_prep_v(c->xc, c->G, c->nrm, c->scal, c->n, c->np, c->dim, c->KP, c->VW,
                                c->V, c->cvec, c->stream));
    // F32: the streamed kernel's operand-ordered column copies (k_swz_f32), or
    // the row-major fp32 copies of the generic tile kernel
    const bool phis = phi_streamed(c);
    const int64_t ntl = (c->n + TBJ_COLS - 1) / TBJ_COLS;
    if (c->dtype == SVGD_F32) {
        if (phis && c->B3)
            HIPCHK(c, launch_swz_b3(mat ? c->zc : c->xc, c->KP, c->V, c->VW, c->cvec, c->n, ntl, c->B3,
                                    c->stream));
        else if (phis)
            HIPCHK(c, launch_swz_f32(mat ? c->zc : c->xc, c->KP, c->V, c->VW, c->cvec, ntl, c->XS,
                                     c->VS, c->stream));
        else
            HIPCHK(c, launch_cvt_f32(c->V, c->np * c->VW, c->Vf, c->stream));
        HIPCHK(c, launch_cvt_f32(c->cvec, c->np, c->cvf, c->stream));
        if (mat) HIPCHK(c, launch_cvt_f32(c->zc, c->np * c->KP, c->zcf, c->stream));
    }
    // level 2: the phi kernel alone (k_phi_rows before its reduce, k_phi_sym,
    // or the tile kernel)
    const bool sym = c->sym && !mat;
    const bool split = c->split_rows && c->in_host_step && c->rowpath && !mat && !sym && opt;
    c->xhalf_ready = split;
    c->n_split += split ? 1 : 0;
    hipEvent_t k0 = sym ? (c->tlevel >= 2 ? take_ev(c) : nullptr) : diag_begin(c, c->stream);
    hipEvent_t k1 = k0 ? take_ev(c) : nullptr;
    if (sym) {
        c->mark = c->phi_end = nullptr;
        SymArgs sa{c->dim,    c->xc,        c->KP,          c->G,        c->nrm,       c->scal,
                   nmax_cur(c),   c->n,         c->sym_nb,      c->sym_u0,   c->sym_u1,    c->srec,
                   c->symok,  c->rowpart,   c->colpart,     c->sym_grid, c->row0,
                   c->nrows,  1.0 / (double)c->n, c->phi, c->rec, c->RS, c->contrib,
                   c->sym_tab, c->sym_tab + 2 * c->sym_nb,
                   c->sym_SM, c->sym_Ia, c->sym_Ib, c->part, c->sym_fS, c->ldp,
                   c->sym_tab + 3 * c->sym_nb, c->sym_qlast, c->tab8k};
        // (when the records' flag says the symmetric form would leave its
        // range, symok = 0, the same launch runs the row stream's work-groups
        // instead; their partials are summed by the finish / k_sym_apply)
        HIPCHK(c, launch_phi_sym(sa, k0, k1, c->stream));
        HIPCHK(c, launch_sym_finish(sa, opt, c->stream));
        if (c->contrib) {
            // every rank's sums of its rows (issued whether or not symok: the
            // ranks' collective sequences must not depend on device data)
            CHK(sym_exchange(c));
            HIPCHK(c, launch_sym_apply(sa, c->contrib + (size_t)c->row0 * (c->dim + 1), c->xrecv_buf, c->xtab_d,
                                       c->xtab_d ? c->world : 1, c->xtab_d ? c->rank : 0, opt, c->stream));
        }
    } else if (c->rowpath && split) {
        // two row halves: the first half's X_{t+1} is final at ev_xhalf, while
        // the second half's phi runs (svgd_step_host_model copies it down and
        // starts its gradient there)
        const int64_t h = c->split_h, d = c->dim;
        OptArgs o1 = *opt, o2 = *opt;
        o2.X += h * d;
        o2.m += h * d;
        o2.v += h * d;
        if (o2.bak) o2.bak += h * d;
        if (o2.xh) o2.xh += h * d;
        HIPCHK(c, launch_phi_rows(c->dim, c->R, c->rec, c->scal, c->row0, h, c->n, c->S2, c->part, h,
                                  1.0 / (double)c->n, nullptr, nullptr, nmax_cur(c), c->phi, &o1, c->stream, k1,
                                  c->phi_kind));
        HIPCHK(c, hipEventRecord(c->ev_xhalf, c->stream));
        hipEvent_t k2 = diag_begin(c, c->stream);
        hipEvent_t k3 = k2 ? take_ev(c) : nullptr;
        HIPCHK(c, launch_phi_rows(c->dim, c->R, c->rec, c->scal, c->row0 + h, c->nrows - h, c->n, c->S2b,
                                  c->part, c->nrows - h, 1.0 / (double)c->n, nullptr, nullptr, nmax_cur(c),
                                  c->phi + h * d, &o2, c->stream, k3, c->phi_kind));
        if (k2) c->ev_diag.push_back({k2, k3, DG_PHI_KERNEL, true});
    } else if (c->rowpath) {
        HIPCHK(c, launch_phi_rows(c->dim, c->R, c->rec, c->scal, c->row0, c->nrows, c->n, c->S, c->part,
                                  c->ldp, 1.0 / (double)c->n, mat ? c->wv : nullptr,
                                  mat ? c->sc_sgn : nullptr, mat ? nullptr : nmax_cur(c), c->phi, opt,
                                  c->stream, k1, mat ? 0 : c->phi_kind));
    } else if (phis)
        HIPCHK(c, c->B3 ? launch_phi_b3(c->KP, c->NCB, c->B3, c->cvf, c->scal, c->row0, c->nrows, ntl,
                                        c->dim, 1.0 / (double)c->n, mat ? c->wv : nullptr, c->xc, c->KP,
                                        c->phi, opt, c->b3_rg, c->stream)
                        : launch_phi_f32s(c->KP, c->NCB, c->XS, c->VS, mat ? c->zcf : c->xcf, c->cvf, c->scal,
                                  c->row0, c->nrows, ntl, c->dim, 1.0 / (double)c->n,
                                  mat ? c->wv : nullptr, c->xc, c->KP, c->phi, opt, c->stream));
    else if (c->dtype == SVGD_F32)
        HIPCHK(c, launch_phi_f32(c->KP, c->NCB, mat ? c->zcf : c->xcf, c->cvf, c->Vf, c->scal,
                                 c->row0, c->nrows, (c->n + TB - 1) / TB, c->n, c->dim,
                                 1.0 / (double)c->n, mat ? c->wv : nullptr, c->xc, c->phi,
                                 c->stream));
    else
        HIPCHK(c, launch_phi(c->KP, c->NCB, mat ? c->zc : c->xc, c->cvec, c->V, c->scal, c->row0,
                             c->nrows, (c->n + TB - 1) / TB, c->n, c->dim, 1.0 / (double)c->n,
                             mat ? c->wv : nullptr, c->phi, c->stream));
    if (k0) {
        if (!c->rowpath) HIPCHK(c, hipEventRecord(k1, c->stream));
        c->ev_diag.push_back({k0, k1, DG_PHI_KERNEL, true});
    }
    if (sym) c->mark = c->phi_end = nullptr;
    if (c->timing) {
        HIPCHK(c, hipEventRecord(ev.b, c->stream));
        c->ev_phi.push_back(ev);
        c->phi_end = c->last_phi_end = ev.b;
    }
    return SVGD_OK;
}

// End of a step's collectives: SVGD_DEBUG_COLL=1 all-gathers every rank's
// hash of the step's collective sequence (communicator, op, count, in issue
// order) and fails unless all are equal -- the cross-rank check of the issue
// order both communicators rely on (svgd_ctx).  Off by default (a blocking
// all-gather per step).
int coll_check_step(svgd_ctx *c)
{
    const uint64_t mine = c->coll_sig;
    c->coll_sig = 0;
    c->coll_phase = 0;
    if (!c->dbg_coll || (!c->comm && !c->hcomm)) return SVGD_OK;
    if (!c->sig_buf) {
        HIPCHK(c, hipMalloc((void **)&c->sig_buf, sizeof(uint64_t) * (size_t)c->world));
    }
    HIPCHK(c, hipMemcpyAsync(c->sig_buf + c->rank, &mine, sizeof(uint64_t), hipMemcpyHostToDevice,
                             c->stream));
    if (c->hcomm) {
        if (hostcomm_allgather(c->hcomm, reinterpret_cast<char *>(c->sig_buf), sizeof(uint64_t),
                               c->stream))
            return fail(c, SVGD_ERR_RCCL, "[RCCL Error] host all-gather failed.");
    } else {
        NCCLCHK(c, ncclAllGather(c->sig_buf + c->rank, c->sig_buf, 1, ncclUint64, c->comm, c->stream));
    }
    std::vector<uint64_t> all((size_t)c->world);
    HIPCHK(c, hipMemcpyAsync(all.data(), c->sig_buf, sizeof(uint64_t) * all.size(),
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->mark = c->phi_end = nullptr;
    for (uint64_t s : all)
        if (s != mine)
            return fail(c, SVGD_ERR_RCCL,
                        "[RCCL Error] ranks issued different collective sequences this step.");
    return SVGD_OK;
}

// This step's optimizer arguments (advances t: call once per step).
int opt_args(svgd_ctx *c, OptArgs *o)
{
    if (c->opt_kind < 0)
        return fail(c, SVGD_ERR_ARG, "[Argument Error] Invalid Optimizer object pointer.");
    c->t += 1;
    double c1 = 1.0, c2 = 1.0;
    if (c->opt_kind == SVGD_OPT_ADAM) {
        c1 = 1.0 - std::pow(c->b1, (double)c->t);
        c2 = 1.0 - std::pow(c->b2, (double)c->t);
    }
    const size_t off = (size_t)c->row0 * c->dim;
    *o = OptArgs{c->opt_kind, c->dim, c->nrows * c->dim, c->m, c->v, c->X + off, c->lr, c->b1,
                 c->b2, c->eps, c1, c2, c->bounded ? c->lower : nullptr,
                 c->bounded ? c->upper : nullptr,
                 // X_t, m_t, v_t of this rank's rows for a redo if the device plan failed
                 c->spec_step ? c->bak : nullptr,
                 // the next host gradient's X_{t+1}
                 c->in_host_step && c->xmirror ? c->h_xm_dev : nullptr};
    return SVGD_OK;
}

// The step's phi and optimizer update: on the row path and the streamed F32
// tile path the phi kernel's epilogue applies it (one launch fewer, no phi
// re-read), else k_opt_update.
int run_phi_opt(svgd_ctx *c)
{
    if (c->opt_kind < 0)
        return fail(c, SVGD_ERR_ARG, "[Argument Error] Invalid Optimizer object pointer.");
    OptArgs o;
    CHK(opt_args(c, &o));
    const bool fused = c->rowpath || phi_streamed(c);
    c->phi_end = nullptr;
    c->xh_valid = false;
    CHK(run_phi(c, fused ? &o : nullptr));
    if (!fused) {
        HIPCHK(c, launch_opt_update(o, c->phi, c->stream));
        c->phi_end = nullptr;
    }
    c->xh_valid = o.xh != nullptr;
    c->xver += 1; // X_{t+1} (the centring fold's version)
    // this rank's rows of X_{t+1} are final here: the next step's X_t copy
    // down (host gradient) need not wait for the X all-gather (P > 1)
    if (c->phi_end) {
        c->ev_xready_use = c->phi_end;
    } else {
        HIPCHK(c, hipEventRecord(c->ev_xready, c->stream));
        c->ev_xready_use = c->ev_xready;
    }
    CHK(allgather_rows(c, c->X));
    c->phi_end = nullptr;
    return coll_check_step(c);
}

int scale_begin(svgd_ctx *c)
{
    if (hipEventQuery(c->ev_scal) != hipSuccess) // the last [a, med] copy has read scal
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_scal, 0));
    const bool med = !(c->scale_method == SVGD_SCALE_FIXED || matrix_scale(c));
    // the median phase's start event goes before the centring (which it
    // needs): an event between two kernels costs a dispatch gap, so the last
    // step's phi end (a timing event) serves when there is one -- the phase
    // then also holds the gap between steps (a diagnostic only: these events
    // feed svgd_get_timing and nothing else)
    if (c->timing && med) {
        EvPair ev = take_pair(c);
        if (c->last_phi_end) {
            ev.spare = ev.a;
            ev.a = c->last_phi_end;
        } else {
            HIPCHK(c, hipEventRecord(ev.a, c->stream));
        }
        c->ev_med.push_back(ev);
    }
    c->last_phi_end = nullptr;
    c->trk_go = false;
    if (med) trk_plan(c);
    if (c->trk_go) {
        const SelState st = make_state(1, &c->trk_lo, c->trk_lo, c->trk_hi);
        CHK(center(c, &st));
    } else {
        CHK(center(c));
    }
    if (med) CHK(median_begin(c));
    c->coll_phase = 1; // every comm call of this phase is issued (upload_g_finish)
    return SVGD_OK;
}

int scale_finish(svgd_ctx *c)
{
    if (c->scale_method == SVGD_SCALE_HESSIAN && !c->hess_ready)
        return fail(c, SVGD_ERR_UNSET,
                    "[Unset Error] Hessian scale: svgd_set_step_hessian_sum was not called this step.");
    if (matrix_scale(c)) {
        c->hess_ready = false;
        return SVGD_OK;
    }
    if (c->scale_method == SVGD_SCALE_FIXED) {
        HIPCHK(c, launch_set_scal(c->fixed_a, NAN, c->scal, c->stream));
        HIPCHK(c, hipEventSynchronize(c->ev_scal)); // no D2H into h_scal pending
        c->h_scal[0] = c->fixed_a;
        c->h_scal[1] = NAN;
        c->scal_fresh = true;
        return SVGD_OK;
    }
    CHK(median_finish(c));
    // a synchronous selection joins the tracking history when resolved
    // (the speculative ones in resolve_pending)
    if (!c->spec_step) c->trk_sync = c->trk_keys ? 1 : 2;
    // [a, med] reach the host only when asked (fetch_scale): no copy on the
    // step's path; the event marks where this step's scale is final (on the
    // speculative path the status event, recorded right after the selection)
    if (c->med_ev_done) {
        c->ev_fin_use = c->ev_status_use;
    } else {
        if (c->timing && !c->ev_med.empty()) HIPCHK(c, hipEventRecord(c->ev_med.back().b, c->stream));
        HIPCHK(c, hipEventRecord(c->ev_fin, c->stream));
        c->ev_fin_use = c->ev_fin;
        c->mark = nullptr;
        CHK(mark_median_end(c));
    }
    c->med_ev_done = false;
    c->scal_fresh = false;
    return SVGD_OK;
}

// [a, med] of the last scale to h_scal (waits for the step's scale only).
int fetch_scale(svgd_ctx *c)
{
    if (c->scal_fresh) return SVGD_OK;
    if (c->status_seq && !c->ev_fin_use) HIPCHK(c, hipStreamSynchronize(c->stream)); // (no scale-final event)
    else HIPCHK(c, hipStreamWaitEvent(c->cstream, c->ev_fin_use ? c->ev_fin_use : c->ev_fin, 0));
    HIPCHK(c, hipMemcpyAsync(c->h_scal, c->scal, 2 * sizeof(double), hipMemcpyDeviceToHost,
                             c->cstream));
    HIPCHK(c, hipEventRecord(c->ev_scal, c->cstream));
    HIPCHK(c, hipEventSynchronize(c->ev_scal));
    c->scal_fresh = true;
    return SVGD_OK;
}

// Check the pending speculative step; on a failed device plan restore X_t,
// m_t, v_t, t and redo the step on the synchronous path (G_t is still on the
// device).  Every rank sees the same status (it derives from all-reduced
// counts), so the redo's collectives match across ranks.
// A synchronous step's selection into the tracking history (its keys are in
// h_trk once the step's scale is final; its bracket counts in h_cnt), or a
// restart of the history when that step selected another way.
int trk_resolve_sync(svgd_ctx *c)
{
    const int s = c->trk_sync;
    c->trk_sync = 0;
    if (s == 0) return SVGD_OK;
    if (s == 2 || !c->trk_allowed) {
        c->trk_n = 0;
        return SVGD_OK;
    }
    HIPCHK(c, hipEventSynchronize(c->ev_fin_use ? c->ev_fin_use : c->ev_fin));
    trk_record(c, c->h_cnt[CNT_LO], c->h_cnt[CNT_HI], c->h_cnt[1]);
    return SVGD_OK;
}

int resolve_pending(svgd_ctx *c)
{
    CHK(trk_resolve_sync(c));
    if (!c->pending) return SVGD_OK;
    c->pending = false;
    if (c->status_seq) {
        // the selection's sequence number in pinned memory (median_finish_spec)
        // Polling: yields for the first 100 us, then 20 us sleeps (the
        // host-gradient threads share the CPUs), and the HIP runtime is asked
        // whether the stream drained at most once per ms, not per iteration
        // (it takes the runtime's locks the gradient worker's HIP calls need;
        // same-box A/B: equal at cfg3 / cfg2, cfg5 6.74-6.92 vs 6.78-7.77 ms
        // with the host gradient's spread 1.58-1.65 vs 1.60-1.97 ms)
        volatile uint64_t *sq = c->h_trk + 8;
        const auto t0 = std::chrono::steady_clock::now();
        auto t_idle = t0, t_query = t0;
        bool idle = false;
        while (*sq != c->status_seq) {
            const auto now = std::chrono::steady_clock::now();
            // the stream has drained and the number is still not there (a
            // bounded grace for the store's visibility): an error, not a hang
            if (!idle && now - t_query > std::chrono::milliseconds(1)) {
                t_query = now;
                if (hipStreamQuery(c->stream) == hipSuccess) {
                    idle = true;
                    t_idle = now;
                }
            }
            if (idle && now - t_idle > std::chrono::milliseconds(200))
                return fail(c, SVGD_ERR_RUNTIME, "[Runtime Error] the selection did not publish its status.");
            if (now - t0 > std::chrono::seconds(300))
                return fail(c, SVGD_ERR_RUNTIME, "[Runtime Error] timed out waiting for the median's status.");
            if (now - t0 < std::chrono::microseconds(100))
                std::this_thread::yield();
            else
                std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
        std::atomic_thread_fence(std::memory_order_acquire);
    } else {
        HIPCHK(c, hipEventSynchronize(c->ev_status_use ? c->ev_status_use : c->ev_status));
    }
    if (*c->h_status == 0) {
        c->last_tot = (int64_t)c->h_trk[7];
        if (c->trk_allowed) trk_record(c, c->h_trk[0], c->h_trk[1], c->h_trk[3]);
        return SVGD_OK;
    }
    if (c->trk_pred >= 0) c->trk_miss += 1;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipStreamSynchronize(c->cstream));
    // this rank's rows of X_t, m_t, v_t back, then X_t all-gathered again
    const size_t sb = sizeof(double) * (size_t)c->nrows * c->dim;
    const size_t cnt = (size_t)c->nrows * c->dim;
    if (c->nrows > 0) {
        HIPCHK(c, hipMemcpyAsync(c->X + (size_t)c->row0 * c->dim, c->bak, sb, hipMemcpyDeviceToDevice,
                                 c->stream));
        HIPCHK(c, hipMemcpyAsync(c->m, c->bak + cnt, sb, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->v, c->bak + 2 * cnt, sb, hipMemcpyDeviceToDevice, c->stream));
    }
    CHK(allgather_rows(c, c->X));
    c->t -= 1;
    c->spec_step = false;
    c->last_fast = false;
    c->xver -= 1; // X_t is back (its centre's partials were never overwritten)
    CHK(scale_begin(c));
    CHK(scale_finish(c));
    CHK(run_phi_opt(c));
    // the redo's selection (synchronous path) continues the tracking history
    return trk_resolve_sync(c);
}

// Speculate this step's median when the last one would have allowed it.
int plan_step(svgd_ctx *c)
{
    // the segment capacity: twice the last selection's keys, a power of two
    // in [CAPR_MIN, CAPG] (a step whose buckets outgrow it fails its plan
    // and is redone synchronously)
    int64_t cap = CAPR_MIN;
    while (cap < 2 * c->last_tot && cap < CAPG) cap <<= 1;
    c->spec_cap = std::min<int64_t>(cap, CAPG);
    c->spec_step = c->spec_allowed && c->last_fast && c->scale_method == SVGD_SCALE_MEDIAN &&
                   c->bucket_cap >= c->spec_cap;
    if (c->spec_step && !c->bak) CHK(dalloc(c, &c->bak, 3 * std::max<int64_t>(1, c->nrows) * c->dim));
    c->n_spec += c->spec_step ? 1 : 0;
    return SVGD_OK;
}

int init_ctx(svgd_ctx *c, int dim, int64_t n, int dtype, int device, int sim_world = 1)
{
    if (dim <= 0 || n <= 0)
        return fail(c, SVGD_ERR_DIM, "[Dimension Error] Particle count and dimension must be positive.");
    if (dtype != SVGD_F64 && dtype != SVGD_F32)
        return fail(c, SVGD_ERR_ARG, "[Argument Error] dtype must be SVGD_F64 or SVGD_F32.");
    const bool f32 = dtype == SVGD_F32;
    if (!pick_tiles(dim, &c->KP, &c->NCB))
        return fail(c, SVGD_ERR_DIM, "[Dimension Error] Device path supports dimension <= 64.");
    // row-stream path (fp64, d <= 16): xc rows are the median records [xc | |xc|^2 | 0..]
    if (dim <= ROWS_MAX_D && !f32) c->KP = med_rec_stride(dim);
    // F32: the phi on the bf16 matrix cores (k_phi_b3) where it applies
    // (SVGD_PHI_B3=0: the fp32-MFMA kernel k_phi_f32s)
    c->want_b3 = false;
    if (f32 && phi_b3_supported(c->KP, c->NCB) && !std::getenv("SVGD_PHI_TILE_GENERIC")) {
        const char *e = std::getenv("SVGD_PHI_B3");
        c->want_b3 = !e || std::atoi(e) != 0;
    }
    // fp64 tiles and the bf16 F32 phi with d = 16 NCB: no V column of ones
    // (row sums on the VALU); SVGD_PHI_S1V=0 keeps the ones column (A/B knob)
    if ((!f32 || c->want_b3) && phi_tile_s1v(dim)) {
        const char *e = std::getenv("SVGD_PHI_S1V");
        if (!e || std::atoi(e) != 0) c->NCB = dim / 16;
    }
    c->dim = dim;
    c->n = n;
    c->dtype = dtype;
    c->device = device;
    c->VW = 16 * c->NCB;
    c->nb = (n + TB - 1) / TB;
    c->np = c->nb * TB + TB;
    c->chunk = (n + c->world - 1) / c->world;
    // svgd_create_sim (measurement only, one rank): run rank 0's share of a
    // P-rank step -- its rows of phi and the optimizer, 1/P of the median's
    // pair tiles with the order statistics' ranks scaled to that share, the
    // host gradient on the threads a rank of P gets -- on one GPU without
    // collectives, to time the per-rank work of a P-GPU run.  The results are
    // NOT the step's (no data from the other ranks): result calls refuse it.
    const int plan_world = c->world == 1 && sim_world > 1 ? sim_world : c->world;
    c->sim_world = plan_world != c->world ? plan_world : 1;
    c->plan_world = plan_world;
    svgd_plan_rows(n, plan_world, c->rank, &c->row0, &c->row1);
    c->nrows = c->row1 - c->row0;
    // k_phi_b3 with one 16-row group per wave, or two (SVGD_PHI_B3_RG=2:
    // half its LDS reads and barriers per MFMA, a measured wash at cfg5 on the
    // power-limited chip, profiles/r06_b3_rg_il_ab.txt)
    if (c->want_b3)
        if (const char *e = std::getenv("SVGD_PHI_B3_RG")) c->b3_rg = std::atoi(e) == 2 ? 2 : 1;
    c->pblock = SVGD_PAIR_BLOCK_DT(dim, dtype);
    c->pnb = (n + c->pblock - 1) / c->pblock;
    c->own_tiles = svgd_plan_pair_tiles(n, c->pblock, plan_world, c->rank);
    {
        const int64_t T = c->pnb * (c->pnb + 1) / 2;
        c->tile0 = T * c->rank / plan_world;
    }
    if (c->sim_world > 1) { // real pairs of the share's tiles (diagonal tiles: upper half)
        for (int64_t t = 0; t < c->own_tiles; ++t) {
            int64_t I, J;
            svgd_plan_pair_tile(n, c->pblock, plan_world, c->rank, t, &I, &J);
            const int64_t ri = std::min<int64_t>(c->pblock, n - I * c->pblock);
            const int64_t rj = std::min<int64_t>(c->pblock, n - J * c->pblock);
            c->sim_pairs += I == J ? ri * (ri - 1) / 2 : ri * rj;
        }
    }
    HIPCHK(c, hipSetDevice(device));
    HIPCHK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPCHK(c, hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
    const int64_t rows_all = c->chunk * c->world;
    CHK(dalloc(c, &c->X, rows_all * dim));
    CHK(dalloc(c, &c->G, rows_all * dim));
    CHK(dalloc(c, &c->xc, c->np * c->KP));
    CHK(dalloc(c, &c->nrm, c->np));
    CHK(dalloc(c, &c->cvec, c->np));
    c->rowpath = dim <= ROWS_MAX_D && !f32;
    if (f32) {
        CHK(dalloc(c, &c->xcf, c->np * c->KP));
        CHK(dalloc(c, &c->nrmf, c->np));
        CHK(dalloc(c, &c->cvf, c->np));
        // KP 32 / 64: the median keys on the bf16 matrix cores (their parts)
        if (const int64_t w = median_key_part_words(c->KP, c->np)) CHK(dalloc(c, &c->XK, w));
    }
    if (c->rowpath) {
        // column splits: enough workgroups to fill every CU at the kernel's occupancy
        int ncu = 256;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess) ncu = prop.multiProcessorCount;
        c->R = dim <= 8 ? 4 : 2; // rows per lane (register budget)
        // 8-wave work-groups, 8192-entry table, columns split over the waves
        // (kind 2); the 4-wave kernel (kind 0) serves the full-matrix scales
        // (signature rows) and an R the 8-wave build does not have
        if (phi_rows_t8k_supported(dim, c->R)) c->phi_kind = 2;
        const int64_t resident = (int64_t)phi_rows_blocks_per_cu(dim, c->R, c->phi_kind) * ncu;
        const int64_t rows_wg = c->phi_kind == 2 ? phi_rows_t8k_rows(c->R) : 256 * (int64_t)c->R;
        const int64_t iblocks = std::max<int64_t>(1, (c->nrows + rows_wg - 1) / rows_wg);
        int64_t S = std::max<int64_t>(1, (resident + iblocks - 1) / iblocks);
        // 2 blocks per resident slot: one block wave per slot left a tail of
        // idle CUs (measured at cfg3, phi launch: S x1 4.00 ms, x2 3.83-3.93,
        // x4 3.81-3.90, x8 3.91-3.95 -- x2 and x4 tie, x2 has half the partials)
        constexpr int split_mult = 2;
        S *= split_mult;
        S = std::min<int64_t>(S, std::max<int64_t>(1, n / 256));
        c->S = (int)S;
        c->RS = phi_rec_stride(dim);
        c->ldp = std::max<int64_t>(1, c->nrows);
        // two row parts (svgd_step_host_model at P > 1, split_rows policy
        // below): the first part's rows get their X_{t+1} while the second
        // part's phi still runs; the second part's gradient has to fit in the
        // next step's median phase.  Each launch takes its own column splits.
        // First part SVGD_PHI_SPLIT_FRAC percent of the rows, default 50
        // (cfg3 8-rank share, profiles/r04_sim_world.jsonl: 50 % 0.632 ms,
        // 62 % 0.783, 72 % 0.765 -- uneven parts made phi itself 40 % slower)
        int frac = 50;
        if (const char *e = std::getenv("SVGD_PHI_SPLIT_FRAC")) frac = std::min(90, std::max(10, std::atoi(e)));
        c->split_h = (c->nrows * frac / 100) / rows_wg * rows_wg;
        if (c->split_h >= c->nrows) c->split_h = 0;
        auto splits = [&](int64_t rows) {
            const int64_t ib = std::max<int64_t>(1, (rows + rows_wg - 1) / rows_wg);
            const int64_t s = std::max<int64_t>(1, (resident + ib - 1) / ib) * split_mult;
            return (int)std::min<int64_t>(s, std::max<int64_t>(1, n / 256));
        };
        if (c->split_h > 0) {
            c->S2 = splits(c->split_h);
            c->S2b = splits(c->nrows - c->split_h);
        }
        CHK(dalloc(c, &c->rec, c->np * c->RS));
        CHK(dalloc(c, &c->xf, c->np * med_f32_stride(dim)));
        CHK(dalloc(c, &c->nmax, 2)); // one slot per X version parity (center)
        CHK(dalloc(c, &c->part, std::max({(int64_t)c->S * c->ldp, (int64_t)c->S2 * c->split_h,
                                          (int64_t)c->S2b * (c->nrows - c->split_h)}) * (dim + 1)));
        // symmetric phi pass: isotropic scales, d <= 8 (a pair feeds two
        // particles).  One rank: default since round 5 from N = 32768 up (with 16-byte record reads
        // cfg3 phi 3.59 -> 3.08 ms, step 4.12 -> 3.68 ms, cfg4 65.5 -> 56.5
        // ms; at cfg2, N = 16384, its extra launches outweigh the saving,
        // 0.200 vs 0.265 ms -- profiles/r05_sym_ab.txt.  SVGD_PHI_SYM=1 / 0
        // forces it on / off)
        // P > 1: rank r runs the units [U r / P, U (r+1) / P), sums every
        // particle's partials from them and a point-to-point exchange hands
        // each rank the pieces of its rows (sym_exchange).  Its phi saving
        // grows as N^2 / P, the exchange as N.  Round 5 (a reduce-scatter of
        // all N (d+1) sums, units not balanced at P = 8): default from N / P >=
        // 16384 (cfg3 shares P = 2 2.008 -> 1.875 ms, P = 4 1.066 -> 1.003, P =
        // 8 0.587 -> 0.582; cfg4 P = 8 7.92 -> 6.84 ms, profiles/r05_sim_sym.txt,
        // r05_cfg4_sim8_sym.txt).  Round 6: the padding-only sub-tiles left out
        // of the units (11 per work-group at cfg3 P = 8 instead of 11 or 12) and
        // ~2.5 MB sent per rank at cfg3 P = 8 instead of 4.1 MB in ring steps:
        // default from N / P >= 8192 (cfg3 at P = 8 included)
        bool want_sym = phi_sym_supported(dim) && n >= 32768 && n / c->plan_world >= 8192;
        int sym_env = -1; // 2 (a test knob): the P > 1 form (sums, reduce-scatter, apply) at any P
        if (const char *e = std::getenv("SVGD_PHI_SYM")) {
            sym_env = std::atoi(e);
            want_sym = phi_sym_supported(dim) && sym_env != 0;
        }
        if (want_sym && phi_sym_geom(dim, &c->symB, &c->symSRS, &c->symNSUB)) {
            const int64_t B = c->symB;
            c->sym_nb = (n + B - 1) / B;
            c->sym_units = svgd_plan_sym_total(n, (int)B, c->symNSUB); // (no padding-only sub-tiles)
            const int64_t Pw = c->plan_world, r = c->sim_world > 1 ? 0 : c->rank;
            const int64_t slots = (int64_t)phi_sym_blocks_per_cu(dim) * ncu;
            const int64_t Vr = c->sym_units * (r + 1) / Pw - c->sym_units * r / Pw;
            c->sym_grid = (int)std::max<int64_t>(1, std::min<int64_t>(Vr, slots));
            // the rank's units, the row blocks each work-group's contiguous run
            // visits and each row block's contiguous row-sum records (plan.cpp)
            const int64_t nbs = c->sym_nb;
            std::vector<int> tab(3 * (size_t)nbs + 2 * (size_t)c->sym_grid);
            int *blkg = tab.data(), *rbase = blkg + 2 * nbs, *wst = rbase + nbs;
            const int64_t nrec = svgd_plan_sym_units(n, (int)B, c->symNSUB, (int)Pw, (int)r, c->sym_grid,
                                                     &c->sym_u0, &c->sym_u1, blkg, rbase, &c->sym_Ia, &c->sym_Ib);
            // each work-group's first unit (the kernel advances from there)
            for (int g = 0; g < c->sym_grid; ++g) {
                const int64_t V = c->sym_u1 - c->sym_u0;
                int64_t t = 0, q = 0;
                svgd_plan_sym_unit(n, (int)B, c->symNSUB, c->sym_u0 + V * g / c->sym_grid, &t, &q);
                wst[2 * g] = (int)t;
                wst[2 * g + 1] = (int)q;
            }
            {
                const int64_t sub = B / c->symNSUB, valid = n - (nbs - 1) * B;
                c->sym_qlast = (int)((valid + sub - 1) / sub);
            }
            c->sym_SM = (nbs - 1) / 2 + 2;
            // the row stream's hand-over inside k_phi_sym (symok = 0): its
            // 8-wave work-groups, one wave of them (<= c->S, the part buffer's splits)
            {
                const int64_t rows_wg = phi_rows_t8k_rows(4);
                const int64_t ib = std::max<int64_t>(1, (c->nrows + rows_wg - 1) / rows_wg);
                c->sym_fS = (int)std::max<int64_t>(1, std::min<int64_t>(c->S, ncu / ib));
            }
            CHK(dalloc(c, &c->sym_tab, (int64_t)tab.size()));
            HIPCHK(c, hipMemcpyAsync(c->sym_tab, tab.data(), tab.size() * sizeof(int), hipMemcpyHostToDevice,
                                     c->stream)); // (after dalloc's memset on the same stream)
            HIPCHK(c, hipStreamSynchronize(c->stream));
            CHK(dalloc(c, &c->srec, c->sym_nb * B * c->symSRS));
            CHK(dalloc(c, &c->rowpart, nrec * B * (dim + 1)));
            // zeroed here once: entries no unit of this rank writes stay zero
            CHK(dalloc(c, &c->colpart, nbs * c->sym_SM * B * (dim + 1)));
            CHK(dalloc(c, &c->symok, 1));
            CHK(dalloc(c, &c->tab8k, 8192));
            HIPCHK(c, launch_fill_tab8k(c->tab8k, c->stream));
            if (Pw > 1 || sym_env == 2) CHK(dalloc(c, &c->contrib, std::max<int64_t>(c->np, c->world * c->chunk) * (dim + 1)));
            if (c->world > 1) {
                // the exchange plan: the same ranges on both sides of every pair of ranks
                c->xsend.assign(2 * (size_t)c->world, 0);
                c->xrecv.assign(3 * (size_t)c->world, 0);
                for (int q = 0; q < c->world; ++q) {
                    int64_t a, b;
                    svgd_plan_sym_exchange(n, (int)B, c->symNSUB, c->world, c->rank, q, &a, &b);
                    c->xsend[2 * q] = a;
                    c->xsend[2 * q + 1] = q == c->rank ? a : b; // (its own rows: not sent)
                    svgd_plan_sym_exchange(n, (int)B, c->symNSUB, c->world, q, c->rank, &a, &b);
                    if (q != c->rank && b > a) {
                        c->xrecv[3 * q] = a;
                        c->xrecv[3 * q + 1] = b;
                        c->xrecv[3 * q + 2] = c->xrecv_rows;
                        c->xrecv_rows += b - a;
                    }
                }
                CHK(dalloc(c, &c->xrecv_buf, std::max<int64_t>(1, c->xrecv_rows) * (dim + 1)));
                HIPCHK(c, hipMalloc((void **)&c->xtab_d, c->xrecv.size() * sizeof(int64_t)));
                HIPCHK(c, hipMemcpy(c->xtab_d, c->xrecv.data(), c->xrecv.size() * sizeof(int64_t),
                                    hipMemcpyHostToDevice));
            }
            c->sym = true;
        }
        // the centring fold (svgd_ctx::cpart)
        c->cpart_stride = (int64_t)center_fold_grid(dim, c->np) * dim;
        CHK(dalloc(c, &c->cpart, 2 * c->cpart_stride));
    } else {
        CHK(dalloc(c, &c->V, c->np * c->VW));
        if (f32) CHK(dalloc(c, &c->Vf, c->np * c->VW));
        if (f32 && phi_f32s_supported(c->KP, c->NCB) && !std::getenv("SVGD_PHI_TILE_GENERIC")) {
            // np is a multiple of 2 TBJ_COLS: ceil(n / TBJ_COLS) tiles fit
            if (c->want_b3) {
                CHK(dalloc(c, &c->B3, (c->np / TBJ_COLS) * phi_b3_tile_words(c->KP, c->NCB)));
            } else {
                CHK(dalloc(c, &c->XS, c->np * c->KP));
                CHK(dalloc(c, &c->VS, c->np * 16 * (c->NCB + 1)));
            }
        }
    }
    CHK(dalloc(c, &c->phi, std::max<int64_t>(1, c->nrows) * dim));
    CHK(dalloc(c, &c->m, std::max<int64_t>(1, c->nrows) * dim));
    CHK(dalloc(c, &c->v, std::max<int64_t>(1, c->nrows) * dim));
    CHK(dalloc(c, &c->lower, dim));
    CHK(dalloc(c, &c->upper, dim));
    CHK(dalloc(c, &c->partial, (int64_t)c->nparts * dim));
    CHK(dalloc(c, &c->scal, 2));
    CHK(dalloc(c, &c->counts, 4 * MAX_COLLECT_BLOCKS)); // <= 4 regions per collect block
    CHK(dalloc(c, &c->below, 4 * MAX_COLLECT_BLOCKS));
    CHK(dalloc(c, &c->cnt3, CNT_LEN + 3));
    CHK(dalloc(c, &c->bpart, (int64_t)MAX_COLLECT_BLOCKS * NBK));
    CHK(dalloc(c, &c->gseg, (int64_t)c->world * (CAPG + 1)));
    if (const char *e = std::getenv("SVGD_BUCKET_CAP")) c->bucket_cap = std::atoll(e);
    if (const char *e = std::getenv("SVGD_MEDIAN_SAMPLE")) c->sample_size = std::max<int64_t>(1, std::atoll(e));
    // A/B and test knob: the reference collect passes (k_pair_rows / k_pair_tiles
    // MODE 0) instead of the matrix-core ones (k_pair_mcol / k_pair_tcol)
    if (const char *e = std::getenv("SVGD_COLLECT_FP64")) c->mcol = std::atoi(e) == 0;
    if (const char *e = std::getenv("SVGD_MCOL_BF16")) c->mcol_bf16 = std::atoi(e) != 0;
    if (c->xf && c->mcol && c->mcol_bf16 && dim <= 8) { // the collect's split-bf16 operands (center)
        CHK(dalloc(c, &c->xsplit, c->np * 8));
        c->collect_blocks = 1280; // k_pair_mcol<D, true>: 5 work-groups per CU (31 KiB LDS, <= 96 VGPRs)
    }
    if (const char *e = std::getenv("SVGD_MEDIAN_SIGMA")) c->bracket_sigma = std::max(0.0, std::atof(e));
    CHK(dalloc(c, &c->st, 1));
    CHK(dalloc(c, &c->ghist, 2 * RADIX));
    CHK(dalloc(c, &c->ccount, 1));
    const size_t hb = sizeof(double) * (size_t)std::max<int64_t>(1, c->nrows) * dim;
    HIPCHK(c, hipHostMalloc((void **)&c->h_x, hb, hipHostMallocDefault));
    HIPCHK(c, hipHostMalloc((void **)&c->h_g, hb, hipHostMallocDefault));
    c->xmirror = hb <= XMIRROR_MAX;
    if (const char *e = std::getenv("SVGD_X_MIRROR")) c->xmirror = std::atoi(e) != 0;
    if (c->xmirror) {
        // coherent: the update epilogue writes it uncached (the host reads it
        // once the step's end event has passed); only a mirroring context pins it
        HIPCHK(c, hipHostMalloc((void **)&c->h_xm, hb, hipHostMallocCoherent));
        HIPCHK(c, hipHostGetDevicePointer((void **)&c->h_xm_dev, c->h_xm, 0));
    }
    HIPCHK(c, hipHostMalloc((void **)&c->h_cnt, (CNT_LEN + 3) * sizeof(unsigned long long),
                            hipHostMallocDefault));
    HIPCHK(c, hipHostMalloc((void **)&c->h_scal, 2 * sizeof(double), hipHostMallocDefault));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_x, hipEventDisableTiming));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_xready, hipEventDisableTiming));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_g, hipEventDisableTiming));
    for (auto &e : c->ev_xch) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_cnt, hipEventDisableTiming));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_scal, hipEventDisableTiming));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_fin, hipEventDisableTiming));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_status, hipEventDisableTiming));
    CHK(dalloc(c, &c->d_status, 1));
    HIPCHK(c, hipHostMalloc((void **)&c->h_status, sizeof(int), hipHostMallocCoherent));
    *c->h_status = 0;
    HIPCHK(c, hipHostGetDevicePointer((void **)&c->h_status_dev, c->h_status, 0));
    HIPCHK(c, hipHostMalloc((void **)&c->h_trk, 16 * sizeof(uint64_t), hipHostMallocCoherent));
    std::memset(c->h_trk, 0, 16 * sizeof(uint64_t));
    HIPCHK(c, hipHostGetDevicePointer((void **)&c->h_trk_dev, c->h_trk, 0));
    if (const char *e = std::getenv("SVGD_SPECULATE")) c->spec_allowed = std::atoi(e) != 0;
    if (const char *e = std::getenv("SVGD_TRACK_BRACKET")) c->trk_allowed = std::atoi(e) != 0;
    if (const char *e = std::getenv("SVGD_TRACK_MIN_WIDTH")) c->trk_min_w = std::atof(e);
    // A miss redoes the step; the band it saves is collect-pass work, which
    // outweighs the misses' cost only when the collect is large: 2.5 x the
    // recent error from N = 32768 up (cfg3: median phase 0.550 -> 0.513 ms,
    // 86 instead of 72 of 90 steps tracked, no miss in 360), 4 below (cfg2
    // at 2.5: 3 misses in 180 steps, slower) -- profiles/r04_track_mult_ab.txt
    c->trk_err_mult = n >= 32768 ? 2.5 : 4.0;
    if (const char *e = std::getenv("SVGD_TRACK_ERR_MULT")) c->trk_err_mult = std::atof(e);
    // half the OpenMP threads, but no more than this rank's share of the
    // cgroup CPU quota (ranks of one node share it; OpenMP sees the affinity
    // mask, not the quota) and at most 32 (the gradient of a 65536-row share
    // takes 0.4 ms on 8 threads, hidden behind the device median).  A
    // measurement context (svgd_create_sim) models rank 0 of a P-GPU node:
    // the pool leases CPUs per GPU (16 with each MI355X), so that rank's
    // share of the node's quota is this one-GPU box's whole quota
    // (SVGD_HOST_THREADS=2 reproduces the 16-CPU box split 8 ways, the
    // pessimistic bound of rounds 3-5).
    {
        int t = std::max(1, omp_get_max_threads() / 2);
        const int q = cgroup_cpus();
        c->cpu_quota = q;
        const int sharing = c->sim_world > 1 ? 1 : std::max(1, c->plan_world);
        if (q > 0) t = std::min(t, std::max(1, q / sharing));
        c->host_threads = std::min(t, 32);
    }
    if (const char *e = std::getenv("SVGD_HOST_THREADS")) c->host_threads = std::max(1, std::atoi(e));
    if (const char *e = std::getenv("SVGD_DEBUG_COLL")) c->dbg_coll = std::atoi(e) != 0;
    // phi in row halves when a rank of 4 or more has more rows per gradient
    // thread than the device's median phase hides: then phi waited for G;
    // with halves the first half's gradient runs beside the second half's
    // phi (cost: a second phi launch and reduce, ~20 us at P = 8).  AVX2
    // gradient block (~18 us per 1000 rows and thread at cfg3's GMM): split
    // above 2048 rows per thread (profiles/r04_sim_world: P = 8 at 2 threads
    // 0.714 -> 0.656 ms).  AVX-512 block (~7 us per 1000 rows and thread on
    // the EPYC 9575F): the whole-rows step wins at P = 8 and 4
    // (profiles/r05_sim_split_ab.txt: 0.580 vs 0.598 ms, 1.052 vs 1.077 ms),
    // split above 8192 rows per thread.
    {
        const int64_t per_thread = svgd_amd::host_grad_avx512() ? 8192 : 2048;
        c->split_rows = c->rowpath && c->split_h > 0 && c->plan_world >= 4 &&
                        c->nrows > per_thread * (int64_t)std::max(1, c->host_threads);
    }
    if (const char *e = std::getenv("SVGD_PHI_SPLIT")) c->split_rows = c->rowpath && c->split_h > 0 && std::atoi(e) != 0;
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_xhalf, hipEventDisableTiming));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return SVGD_OK;
}

} // namespace

extern "C" {

int svgd_get_unique_id(void *unique_id128)
{
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return SVGD_ERR_RCCL;
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    std::memcpy(unique_id128, &id, sizeof(id));
    return SVGD_OK;
}

int svgd_create(svgd_ctx **out, int dim, int64_t n, int dtype, int device)
{
    if (!out) return SVGD_ERR_ARG;
    svgd_ctx *c = new svgd_ctx();
    *out = c;
    return init_ctx(c, dim, n, dtype, device);
}

int svgd_create_sim(svgd_ctx **out, int dim, int64_t n, int dtype, int device, int sim_world)
{
    if (!out) return SVGD_ERR_ARG;
    svgd_ctx *c = new svgd_ctx();
    *out = c;
    if (sim_world < 1) return fail(c, SVGD_ERR_ARG, "[Argument Error] Invalid simulated world size.");
    return init_ctx(c, dim, n, dtype, device, sim_world);
}

int svgd_create_dist(svgd_ctx **out, int dim, int64_t n, int dtype, int device, int world,
                     int rank, const void *unique_id128)
{
    if (!out) return SVGD_ERR_ARG;
    svgd_ctx *c = new svgd_ctx();
    *out = c;
    if (world < 1 || rank < 0 || rank >= world ||
        (world > 1 && !unique_id128 && !std::getenv("SVGD_HOSTCOMM")))
        return fail(c, SVGD_ERR_ARG, "[Argument Error] Invalid world/rank.");
    c->world = world;
    c->rank = rank;
    CHK(init_ctx(c, dim, n, dtype, device));
    if (world > 1 && std::getenv("SVGD_HOSTCOMM")) {
        // rehearsal backend: ranks sharing one GPU, collectives through host shm
        const size_t slot = std::max<size_t>(
            std::max<size_t>(
                std::max<size_t>((size_t)c->chunk * c->dim, (size_t)c->dim * c->dim) * sizeof(double),
                2 * RADIX * sizeof(unsigned long long)),
            std::max<size_t>((CAPG + 1) * sizeof(uint64_t), (3 + NBK) * sizeof(uint64_t)));
        const size_t slot_rs = c->contrib ? 2 * sizeof(int64_t) * (size_t)world +
                                                (size_t)c->n * (c->dim + 1) * sizeof(double)
                                          : 0;
        if (hostcomm_create(&c->hcomm, std::getenv("SVGD_HOSTCOMM"), world, rank, std::max(slot, slot_rs)))
            return fail(c, SVGD_ERR_RCCL, "[RCCL Error] host communicator setup failed.");
        return SVGD_OK;
    }
    // world == 1 with a unique id: a one-rank RCCL communicator, so every
    // collective of the sharded step runs through RCCL on a single GPU
    if (unique_id128) {
        ncclUniqueId id;
        std::memcpy(&id, unique_id128, sizeof(id));
        NCCLCHK(c, ncclCommInitRank(&c->comm, world, id, rank));
        // the G all-gather's own communicator and stream (upload_g_finish):
        // by default at P >= 2, so the all-gather of G runs beside the median
        // (15-30 us off the P = 8 critical path); SVGD_G_COMM=0 /
        // 1 on every rank forces it off / on (the split is collective).
        // Every rank learns whether every split succeeded (a min all-reduce
        // over comm): one rank gathering G on gcomm while another gathers it
        // on comm would hang both, so any failure drops gcomm everywhere and
        // the G all-gather stays on the compute stream.
        bool want_g = world > 1;
        if (const char *e = std::getenv("SVGD_G_COMM")) want_g = std::atoi(e) != 0;
        if (want_g) {
            int ok = ncclCommSplit(c->comm, 0, rank, &c->gcomm, nullptr) == ncclSuccess && c->gcomm;
            if (ok && hipStreamCreateWithFlags(&c->gstream, hipStreamNonBlocking) != hipSuccess) ok = 0;
            if (ok && hipEventCreateWithFlags(&c->ev_gg, hipEventDisableTiming) != hipSuccess) ok = 0;
            int *d_ok = nullptr;
            HIPCHK(c, hipMalloc((void **)&d_ok, sizeof(int)));
            HIPCHK(c, hipMemcpy(d_ok, &ok, sizeof(int), hipMemcpyHostToDevice));
            NCCLCHK(c, ncclAllReduce(d_ok, d_ok, 1, ncclInt32, ncclMin, c->comm, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            HIPCHK(c, hipMemcpy(&ok, d_ok, sizeof(int), hipMemcpyDeviceToHost));
            (void)hipFree(d_ok);
            if (!ok) {
                if (c->gcomm) (void)ncclCommDestroy(c->gcomm);
                c->gcomm = nullptr;
            }
        }
    }
    return SVGD_OK;
}

int svgd_destroy(svgd_ctx *c)
{
    if (!c) return SVGD_OK;
    c->worker.reset(); // idle between steps: joins the gradient thread
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->cstream) (void)hipStreamSynchronize(c->cstream);
    if (c->gstream) (void)hipStreamSynchronize(c->gstream);
    if (c->gcomm) (void)ncclCommDestroy(c->gcomm);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    if (c->hcomm) hostcomm_destroy(c->hcomm);
    double *dbufs[] = {c->X,     c->G,     c->xc,      c->nrm,  c->cvec, c->V,   c->phi,
                       c->m,     c->v,     c->lower,   c->upper, c->partial, c->scal, c->rec,
                       c->part,  c->dm_mu, c->dm_prec, c->sc_src, c->sc_M, c->sc_L, c->wv, c->zc,
                       c->sc_sgn,  c->sc_work, c->bak, c->srec, c->rowpart, c->colpart, c->contrib,
                       c->xrecv_buf, c->tab8k};
    float *fbufs[] = {c->xcf, c->nrmf, c->cvf, c->Vf, c->zcf, c->XS, c->VS};
    for (float *p : fbufs)
        if (p) (void)hipFree(p);
    if (c->B3) (void)hipFree(c->B3);
    if (c->XK) (void)hipFree(c->XK);
    if (c->cpart) (void)hipFree(c->cpart);
    for (double *p : dbufs)
        if (p) (void)hipFree(p);
    void *obufs[] = {c->sample_keys, c->regions, c->counts, c->below, c->cnt3, c->st, c->ghist,
                     c->xf,          c->nmax,    c->sc_err, c->cbuf, c->ccount, c->d_status,
                     c->bpart,       c->gseg, c->symok, c->sym_tab, c->xtab_d, c->xsplit};
    for (void *p : obufs)
        if (p) (void)hipFree(p);
    void *hbufs[] = {c->h_x, c->h_g, c->h_xm, c->h_cnt, c->h_scal, c->h_err, c->h_status, c->h_trk};
    for (void *p : hbufs)
        if (p) (void)hipHostFree(p);
    for (auto *v : {&c->ev_phi, &c->ev_med, &c->ev_pool})
        for (auto &e : *v) {
            (void)hipEventDestroy(e.spare ? e.spare : e.a); // (a shared mark is ev_med's b)
            (void)hipEventDestroy(e.b);
        }
    if (c->ev_x) (void)hipEventDestroy(c->ev_x);
    if (c->ev_xready) (void)hipEventDestroy(c->ev_xready);
    if (c->ev_g) (void)hipEventDestroy(c->ev_g);
    for (auto &e : c->ev_xch)
        if (e) (void)hipEventDestroy(e);
    if (c->ev_cnt) (void)hipEventDestroy(c->ev_cnt);
    if (c->ev_scal) (void)hipEventDestroy(c->ev_scal);
    if (c->ev_fin) (void)hipEventDestroy(c->ev_fin);
    if (c->ev_status) (void)hipEventDestroy(c->ev_status);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->cstream) (void)hipStreamDestroy(c->cstream);
    if (c->gstream) (void)hipStreamDestroy(c->gstream);
    if (c->ev_gg) (void)hipEventDestroy(c->ev_gg);
    if (c->ev_xhalf) (void)hipEventDestroy(c->ev_xhalf);
    for (auto &e : c->ev_diag) {
        if (e.own_a) (void)hipEventDestroy(e.a);
        (void)hipEventDestroy(e.b);
    }
    for (hipEvent_t e : c->ev_single) (void)hipEventDestroy(e);
    delete c;
    return SVGD_OK;
}

const char *svgd_last_error(const svgd_ctx *c) { return c ? c->err.c_str() : "SVGDCpp: null context"; }

int svgd_shard(const svgd_ctx *c, int64_t *row0, int64_t *row1)
{
    if (!c) return SVGD_ERR_ARG;
    if (row0) *row0 = c->row0;
    if (row1) *row1 = c->row1;
    return SVGD_OK;
}

int svgd_set_optimizer(svgd_ctx *c, int kind, double lr, double beta1, double beta2, double eps)
{
    if (!c) return SVGD_ERR_ARG;
    CHK(resolve_pending(c));
    if (kind == SVGD_OPT_ADAM && (beta1 >= 1.0 || beta1 < 0.0 || beta2 >= 1.0 || beta2 < 0.0))
        return fail(c, SVGD_ERR_ARG, "[Argument Error] Invalid value for decay parameter beta.");
    if (kind == SVGD_OPT_RMSPROP && (beta1 > 1.0 || beta1 < 0.0))
        return fail(c, SVGD_ERR_ARG, "[Argument Error] Invalid value for decay parameter beta.");
    if (kind < SVGD_OPT_ADAM || kind > SVGD_OPT_RMSPROP)
        return fail(c, SVGD_ERR_ARG, "[Argument Error] Invalid Optimizer object pointer.");
    c->opt_kind = kind;
    c->lr = lr;
    c->b1 = beta1;
    c->b2 = beta2;
    c->eps = eps;
    return svgd_reset_optimizer(c);
}

int svgd_reset_optimizer(svgd_ctx *c)
{
    if (!c) return SVGD_ERR_ARG;
    CHK(resolve_pending(c));
    HIPCHK(c, hipSetDevice(c->device));
    const size_t bytes = sizeof(double) * (size_t)std::max<int64_t>(1, c->nrows) * c->dim;
    HIPCHK(c, hipMemsetAsync(c->m, 0, bytes, c->stream));
    HIPCHK(c, hipMemsetAsync(c->v, 0, bytes, c->stream));
    c->t = 0;
    return SVGD_OK;
}

int svgd_set_bounds(svgd_ctx *c, const double *lower, const double *upper)
{
    if (!c) return SVGD_ERR_ARG;
    CHK(resolve_pending(c));
    if (!lower && !upper) {
        c->bounded = false;
        return SVGD_OK;
    }
    if (!lower || !upper)
        return fail(c, SVGD_ERR_DIM, "[Dimension Error] The provided bounds have incorrect dimensions.");
    HIPCHK(c, hipMemcpy(c->lower, lower, sizeof(double) * c->dim, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->upper, upper, sizeof(double) * c->dim, hipMemcpyHostToDevice));
    c->bounded = true;
    return SVGD_OK;
}

int alloc_matrix_scale(svgd_ctx *c)
{
    if (c->sc_M) return SVGD_OK;
    const int64_t dd = (int64_t)c->dim * c->dim;
    CHK(dalloc(c, &c->sc_src, dd));
    CHK(dalloc(c, &c->sc_M, dd));
    CHK(dalloc(c, &c->sc_L, dd));
    CHK(dalloc(c, &c->sc_sgn, c->dim));
    CHK(dalloc(c, &c->sc_work, 2 * dd));
    CHK(dalloc(c, &c->wv, c->np * c->dim));
    if (!c->rowpath) CHK(dalloc(c, &c->zc, c->np * c->KP));
    if (c->dtype == SVGD_F32) CHK(dalloc(c, &c->zcf, c->np * c->KP));
    CHK(dalloc(c, &c->sc_err, 1));
    HIPCHK(c, hipHostMalloc((void **)&c->h_err, sizeof(int), hipHostMallocDefault));
    *c->h_err = 0;
    return SVGD_OK;
}

int svgd_set_scale(svgd_ctx *c, int method, double fixed_a)
{
    if (!c) return SVGD_ERR_ARG;
    CHK(resolve_pending(c));
    if (method != SVGD_SCALE_MEDIAN && method != SVGD_SCALE_FIXED && method != SVGD_SCALE_HESSIAN)
        return fail(c, SVGD_ERR_ARG, "[Argument error] Invalid scale method Enum provided.");
    if (method == SVGD_SCALE_HESSIAN) CHK(alloc_matrix_scale(c));
    c->scale_method = method;
    c->fixed_a = fixed_a;
    c->hess_ready = false;
    return SVGD_OK;
}

int svgd_set_scale_matrix(svgd_ctx *c, const double *M)
{
    if (!c || !M) return c ? fail(c, SVGD_ERR_ARG, "[Argument Error] Null scale matrix.") : SVGD_ERR_ARG;
    const int d = c->dim;
    for (int r = 0; r < d; ++r)
        for (int q = 0; q < r; ++q)
            if (M[r * d + q] != M[q * d + r])
                return fail(c, SVGD_ERR_ARG, "[Argument Error] The kernel scale matrix must be symmetric.");
    CHK(resolve_pending(c));
    CHK(alloc_matrix_scale(c));
    HIPCHK(c, hipMemcpyAsync(c->sc_src, M, sizeof(double) * (size_t)d * d, hipMemcpyHostToDevice,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->scale_method = SVGD_SCALE_MATRIX;
    return SVGD_OK;
}

int svgd_set_step_hessian_sum(svgd_ctx *c, const double *H_shard_sum)
{
    if (!c || !H_shard_sum) return c ? fail(c, SVGD_ERR_ARG, "[Argument Error] Null Hessian sum.") : SVGD_ERR_ARG;
    CHK(resolve_pending(c));
    if (c->scale_method != SVGD_SCALE_HESSIAN)
        return fail(c, SVGD_ERR_ARG, "[Argument Error] The kernel scale method is not Hessian.");
    const size_t dd = (size_t)c->dim * c->dim;
    c->h_mat.assign(H_shard_sum, H_shard_sum + dd);
    HIPCHK(c, hipMemcpyAsync(c->sc_src, c->h_mat.data(), sizeof(double) * dd, hipMemcpyHostToDevice,
                             c->stream));
    CHK(allreduce_f64(c, c->sc_src, dd));
    HIPCHK(c, hipStreamSynchronize(c->stream)); // h_mat may be reused
    c->hess_ready = true;
    return SVGD_OK;
}

int svgd_get_scale_matrix(svgd_ctx *c, double *M_out)
{
    if (!c || !M_out) return SVGD_ERR_ARG;
    CHK(resolve_pending(c));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const int d = c->dim;
    if (matrix_scale(c)) {
        if (*c->h_err == 1)
            return fail(c, SVGD_ERR_RUNTIME, "[Runtime Error] The kernel scale matrix is not finite.");
        if (*c->h_err == 2 && !c->rowpath)
            return fail(c, SVGD_ERR_RUNTIME,
                        "[Runtime Error] The kernel scale matrix is indefinite; the device path "
                        "supports indefinite matrices for fp64 particles with d <= 16 only.");
        HIPCHK(c, hipMemcpy(M_out, c->sc_M, sizeof(double) * (size_t)d * d, hipMemcpyDeviceToHost));
        return SVGD_OK;
    }
    CHK(fetch_scale(c));
    const double a = c->scale_method == SVGD_SCALE_FIXED ? c->fixed_a : c->h_scal[0];
    for (int r = 0; r < d; ++r)
        for (int q = 0; q < d; ++q) M_out[r * d + q] = r == q ? a : 0.0;
    return SVGD_OK;
}

int svgd_set_particles(svgd_ctx *c, const double *X)
{
    if (!c || !X) return SVGD_ERR_ARG;
    CHK(resolve_pending(c));
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(c->X, X, sizeof(double) * (size_t)c->n * c->dim,
                             hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipEventRecord(c->ev_xready, c->stream));
    c->ev_xready_use = c->ev_xready;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->have_particles = true;
    c->xhalf_ready = false;
    c->xh_valid = false;
    c->xver += 1;
    c->cpart_ver[0] = c->cpart_ver[1] = -1; // new particles: centred on their own mean
    c->trk_n = c->trk_nerr = c->trk_nerrc = 0; // new particles: the median history restarts
    return SVGD_OK;
}

int svgd_get_particles(svgd_ctx *c, double *X)
{
    CHK(check_results(c));
    CHK(resolve_pending(c));
    if (!X) return fail(c, SVGD_ERR_ARG, "[Argument Error] Null output buffer.");
    HIPCHK(c, hipMemcpyAsync(X, c->X, sizeof(double) * (size_t)c->n * c->dim,
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return SVGD_OK;
}

int svgd_get_shard(svgd_ctx *c, double *X_shard)
{
    CHK(check_results(c));
    CHK(resolve_pending(c));
    if (c->nrows == 0) return SVGD_OK;
    HIPCHK(c, hipMemcpyAsync(X_shard, c->X + (size_t)c->row0 * c->dim,
                             sizeof(double) * (size_t)c->nrows * c->dim, hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return SVGD_OK;
}

int svgd_median_scale(svgd_ctx *c, double *a_out, double *med_out)
{
    CHK(check_results(c));
    CHK(resolve_pending(c));
    c->spec_step = false;
    const int keep = c->scale_method;
    c->scale_method = SVGD_SCALE_MEDIAN;
    int rc = scale_begin(c);
    if (rc == SVGD_OK) rc = scale_finish(c);
    c->scale_method = keep;
    c->trk_sync = 0; // not a step: X_t's median would enter the history twice
    c->coll_phase = 0;
    CHK(rc);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    CHK(fetch_scale(c));
    if (a_out) *a_out = c->h_scal[0];
    if (med_out) *med_out = c->h_scal[1];
    return SVGD_OK;
}

int svgd_phi(svgd_ctx *c, const double *G_shard, double a, double *phi_out)
{
    CHK(check_results(c));
    CHK(resolve_pending(c));
    c->spec_step = false;
    if (hipEventQuery(c->ev_scal) != hipSuccess) // the last [a, med] copy has read scal
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_scal, 0));
    CHK(center(c));
    HIPCHK(c, launch_set_scal(a, NAN, c->scal, c->stream));
    // the host copy of [a, med] follows (svgd_last_scale after svgd_phi)
    HIPCHK(c, hipEventSynchronize(c->ev_scal)); // no D2H into h_scal pending
    c->h_scal[0] = a;
    c->h_scal[1] = NAN;
    c->scal_fresh = true;
    CHK(upload_g(c, G_shard));
    CHK(run_phi(c, nullptr));
    if (phi_out && c->nrows > 0) {
        HIPCHK(c, hipMemcpyAsync(phi_out, c->phi, sizeof(double) * (size_t)c->nrows * c->dim,
                                 hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return SVGD_OK;
}

int svgd_begin_step(svgd_ctx *c, double *X_shard_out)
{
    CHK(check_ready(c));
    CHK(resolve_pending(c));
    if (c->opt_kind < 0)
        return fail(c, SVGD_ERR_ARG, "[Argument Error] Invalid Optimizer object pointer.");
    const size_t bytes = sizeof(double) * (size_t)c->nrows * c->dim;
    if (X_shard_out && c->nrows > 0) {
        // X_t is final once the previous step's update (and all-gather) ran
        HIPCHK(c, hipStreamWaitEvent(c->cstream, c->ev_xready_use ? c->ev_xready_use : c->ev_xready, 0));
        HIPCHK(c, hipMemcpyAsync(c->h_x, c->X + (size_t)c->row0 * c->dim, bytes,
                                 hipMemcpyDeviceToHost, c->cstream));
        HIPCHK(c, hipEventRecord(c->ev_x, c->cstream));
    }
    CHK(plan_step(c));
    CHK(scale_begin(c));
    if (X_shard_out && c->nrows > 0) {
        HIPCHK(c, hipEventSynchronize(c->ev_x));
        if (X_shard_out != c->h_x) std::memcpy(X_shard_out, c->h_x, bytes);
    }
    return SVGD_OK;
}

int svgd_finish_step(svgd_ctx *c, const double *G_shard)
{
    CHK(check_ready(c));
    if (c->coll_phase != 1) // (also keeps the collectives in their order, svgd_ctx)
        return fail(c, SVGD_ERR_RUNTIME, "[Runtime Error] svgd_finish_step without svgd_begin_step.");
    CHK(upload_g_begin(c, G_shard));
    // the G all-gather is queued before the host waits for the median counts
    // (scale_finish), so the device runs it during that round trip
    CHK(upload_g_finish(c));
    CHK(scale_finish(c));
    CHK(run_phi_opt(c));
    return SVGD_OK;
}

int svgd_step_host_model(svgd_ctx *c, const void *model)
{
    CHK(check_ready(c));
    const svgd_amd::HostModel *m = static_cast<const svgd_amd::HostModel *>(model);
    if (!m || m->d != c->dim)
        return fail(c, SVGD_ERR_ARG, "[Argument Error] Host model missing or of another dimension.");
    if (c->scale_method == SVGD_SCALE_HESSIAN) // (the split calls carry the caller's sum)
        return fail(c, SVGD_ERR_UNSET,
                    "[Unset Error] Hessian scale: svgd_set_step_hessian_sum was not called this step "
                    "(svgd_step_host_model does not supply it; use svgd_begin_step / "
                    "svgd_set_step_hessian_sum / svgd_finish_step).");
    CHK(resolve_pending(c));
    if (c->opt_kind < 0)
        return fail(c, SVGD_ERR_ARG, "[Argument Error] Invalid Optimizer object pointer.");
    const int d = c->dim;
    const int64_t rows = c->nrows;
    // row chunks of >= 1 MiB (a chunk's copy, event and OpenMP region cost
    // ~10 us: smaller chunks lose more than they overlap), at most XCH
    const int64_t min_rows = std::max<int64_t>(1, (int64_t(1) << 20) / (8 * d));
    // the last step ran phi in row halves: the first half's chunks wait for
    // its X_{t+1} only (ev_xhalf), so their gradient starts while the second
    // half's phi still runs; chunks never straddle the halves
    const int64_t hsplit = c->xhalf_ready ? c->split_h : 0;
    const int nh = hsplit > 0 ? (int)std::max<int64_t>(1, std::min<int64_t>(XCH / 2, hsplit / min_rows)) : 0;
    const int nch = hsplit > 0 ? 2 * nh
                               : (int)std::max<int64_t>(1, std::min<int64_t>(XCH, rows / min_rows));
    auto chunk = [hsplit, nh, nch, rows](int q, int64_t *r0, int64_t *r1) {
        if (hsplit > 0) {
            const int64_t b = q < nh ? 0 : hsplit, len = q < nh ? hsplit : rows - hsplit;
            const int qq = q < nh ? q : q - nh;
            *r0 = b + len * qq / nh;
            *r1 = b + len * (qq + 1) / nh;
            return;
        }
        *r0 = rows * q / nch;
        *r1 = rows * (q + 1) / nch;
    };
    HIPCHK(c, hipEventSynchronize(c->ev_g)); // the previous step's upload has left h_g
    // the event chunk q's X_t waits for: its copy's, or -- when the last
    // update stored X_t into h_x (xh_valid) -- that update's own end
    hipEvent_t xwait[XCH];
    if (rows > 0) {
        // X_t is final once the previous step's update (and all-gather) ran
        hipEvent_t xev = c->ev_xready_use ? c->ev_xready_use : c->ev_xready;
        if (c->xh_valid) {
            for (int q = 0; q < nch; ++q) xwait[q] = hsplit > 0 && q < nh ? c->ev_xhalf : xev;
        } else {
            HIPCHK(c, hipStreamWaitEvent(c->cstream, hsplit > 0 ? c->ev_xhalf : xev, 0));
            for (int q = 0; q < nch; ++q) {
                int64_t r0, r1;
                chunk(q, &r0, &r1);
                if (hsplit > 0 && q == nh) HIPCHK(c, hipStreamWaitEvent(c->cstream, xev, 0));
                HIPCHK(c, hipMemcpyAsync(c->h_x + r0 * d, c->X + (size_t)(c->row0 + r0) * d,
                                         sizeof(double) * (size_t)(r1 - r0) * d, hipMemcpyDeviceToHost,
                                         c->cstream));
                HIPCHK(c, hipEventRecord(c->ev_xch[q], c->cstream));
                xwait[q] = c->ev_xch[q];
            }
        }
    }
    // the gradient's input: X_t from the last update's mirror, or its copy
    const double *hx = c->xh_valid ? c->h_xm : c->h_x;
    c->n_mirror += c->xh_valid && rows > 0 ? 1 : 0;
    // the gradient thread: each chunk waits for its X_t copy, evaluates the
    // model and queues its G copy on the copy stream (the calling thread only
    // touches `stream` until it waits for this job)
    if (!c->worker) c->worker.reset(new HostWorker());
    using clk = std::chrono::steady_clock;
    auto ms_since = [](clk::time_point t0, clk::time_point t1) {
        return std::chrono::duration<double, std::milli>(t1 - t0).count();
    };
    const clk::time_point t_post = clk::now();
    std::array<hipEvent_t, XCH> xw;
    std::copy(xwait, xwait + (rows > 0 ? nch : 0), xw.begin());
    c->worker->post([c, m, d, rows, nch, chunk, ms_since, t_post, xw, hx](std::string &msg) -> int {
        for (int q = 0; q < nch && rows > 0; ++q) {
            int64_t r0, r1;
            chunk(q, &r0, &r1);
            const clk::time_point tw = clk::now();
            hipError_t e = hipEventSynchronize(xw[q]);
            if (e != hipSuccess) {
                msg = std::string("SVGDCpp: [HIP Error] X_t chunk copy: ") + hipGetErrorString(e);
                return SVGD_ERR_HIP;
            }
            const clk::time_point tg = clk::now();
            if (const int rc = model_logp_grad_threads(m, hx + r0 * d, r1 - r0, c->h_g + r0 * d,
                                                       c->host_threads)) {
                msg = rc == SVGD_ERR_RUNTIME ? "SVGDCpp: [Runtime Error] Host model evaluation: out of memory."
                                             : "SVGDCpp: [Argument Error] Host model evaluation failed.";
                return rc;
            }
            c->h_xwait_ms += ms_since(tw, tg);
            c->h_grad_ms += ms_since(tg, clk::now());
            e = hipMemcpyAsync(c->G + (size_t)(c->row0 + r0) * d, c->h_g + r0 * d,
                               sizeof(double) * (size_t)(r1 - r0) * d, hipMemcpyHostToDevice,
                               c->cstream);
            if (e != hipSuccess) {
                msg = std::string("SVGDCpp: [HIP Error] G chunk copy: ") + hipGetErrorString(e);
                return SVGD_ERR_HIP;
            }
        }
        hipError_t e = hipEventRecord(c->ev_g, c->cstream);
        // the gradient thread waits for its copies to land (the device is
        // still in the median): the compute stream then needs no barrier on
        // the copy stream (upload_g_finish)
        if (e == hipSuccess) e = hipEventSynchronize(c->ev_g);
        if (e != hipSuccess) {
            msg = std::string("SVGDCpp: [HIP Error] G event: ") + hipGetErrorString(e);
            return SVGD_ERR_HIP;
        }
        c->h_job_ms += ms_since(t_post, clk::now());
        return SVGD_OK;
    });
    int rc = plan_step(c);
    if (rc == SVGD_OK) rc = scale_begin(c);
    std::string wmsg;
    const clk::time_point tw0 = clk::now();
    const int wrc = c->worker->wait(wmsg); // always joined before returning
    c->h_wait_ms += ms_since(tw0, clk::now());
    c->h_steps += 1;
    CHK(rc);
    if (wrc != SVGD_OK) {
        c->err = wmsg;
        return wrc;
    }
    CHK(upload_g_finish(c));
    CHK(scale_finish(c));
    c->in_host_step = true;
    rc = run_phi_opt(c);
    c->in_host_step = false;
    return rc;
}

int svgd_step(svgd_ctx *c, const double *G_shard)
{
    if (G_shard) {
        CHK(svgd_begin_step(c, nullptr));
        return svgd_finish_step(c, G_shard);
    }
    // fully device-resident step: grad log p from the device model
    CHK(check_ready(c));
    if (c->dm_k == 0)
        return fail(c, SVGD_ERR_ARG,
                    "[Argument Error] Null log-gradient buffer and no device model set.");
    CHK(svgd_begin_step(c, nullptr));
    HIPCHK(c, launch_gauss_grad(c->X + (size_t)c->row0 * c->dim, c->nrows, c->dim, c->dm_k,
                                c->dm_mu, c->dm_prec, c->G + (size_t)c->row0 * c->dim, c->stream));
    c->mark = nullptr; // (the gradient kernel runs after the median's end event)
    CHK(scale_finish(c));
    CHK(allgather_rows(c, c->G));
    CHK(run_phi_opt(c));
    return SVGD_OK;
}

int svgd_set_device_model(svgd_ctx *c, const void *model)
{
    if (!c) return SVGD_ERR_ARG;
    CHK(resolve_pending(c));
    if (!model) {
        c->dm_k = 0;
        return SVGD_OK;
    }
    const HostModel *m = static_cast<const HostModel *>(model);
    if (m->d != c->dim)
        return fail(c, SVGD_ERR_DIM, "[Dimension Error] Model dimension does not match the particles.");
    if (m->d > 64)
        return fail(c, SVGD_ERR_ARG, "[Argument Error] Device model supports d <= 64.");
    CHK(dalloc(c, &c->dm_mu, (int64_t)m->k * m->d));
    CHK(dalloc(c, &c->dm_prec, (int64_t)m->k * m->d * m->d));
    HIPCHK(c, hipMemcpyAsync(c->dm_mu, m->mu.data(), sizeof(double) * m->mu.size(),
                             hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->dm_prec, m->prec.data(), sizeof(double) * m->prec.size(),
                             hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->dm_k = m->k;
    return SVGD_OK;
}

int svgd_device_logp_grad(svgd_ctx *c, double *G_shard_out)
{
    CHK(check_ready(c));
    CHK(resolve_pending(c));
    if (c->dm_k == 0) return fail(c, SVGD_ERR_UNSET, "[Unset Error] No device model set.");
    if (!G_shard_out) return fail(c, SVGD_ERR_ARG, "[Argument Error] Null output buffer.");
    HIPCHK(c, launch_gauss_grad(c->X + (size_t)c->row0 * c->dim, c->nrows, c->dim, c->dm_k,
                                c->dm_mu, c->dm_prec, c->phi, c->stream));
    HIPCHK(c, hipMemcpyAsync(G_shard_out, c->phi, sizeof(double) * (size_t)c->nrows * c->dim,
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return SVGD_OK;
}

int svgd_host_buffers(svgd_ctx *c, double **x_shard, double **g_shard)
{
    if (!c) return SVGD_ERR_ARG;
    if (x_shard) *x_shard = c->h_x;
    if (g_shard) *g_shard = c->h_g;
    return SVGD_OK;
}

int svgd_sync(svgd_ctx *c)
{
    if (!c) return SVGD_ERR_ARG;
    CHK(resolve_pending(c));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return SVGD_OK;
}

int svgd_last_scale(const svgd_ctx *c, double *a_out, double *med_out, int *path)
{
    if (!c) return SVGD_ERR_ARG;
    svgd_ctx *m = const_cast<svgd_ctx *>(c);
    CHK(resolve_pending(m));
    CHK(fetch_scale(m));
    if (a_out) *a_out = c->h_scal[0];
    if (med_out) *med_out = c->h_scal[1];
    if (path) *path = c->last_path;
    return SVGD_OK;
}

int svgd_last_median_keys(svgd_ctx *c, double *sq_lo, double *sq_hi, int64_t *rank_lo,
                          int64_t *rank_hi)
{
    if (!c) return SVGD_ERR_ARG;
    CHK(resolve_pending(c));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    SelState s;
    HIPCHK(c, hipMemcpy(&s, c->st, sizeof(SelState), hipMemcpyDeviceToHost));
    int64_t rlo, rhi;
    svgd_plan_median_ranks(c->n, &rlo, &rhi);
    auto val = [&](int src) {
        if (src < 0) return 0.0;
        double v;
        std::memcpy(&v, &s.prefix[src], sizeof(v));
        return v;
    };
    if (sq_lo) *sq_lo = val(c->src_lo);
    if (sq_hi) *sq_hi = val(c->src_hi);
    if (rank_lo) *rank_lo = rlo;
    if (rank_hi) *rank_hi = rhi;
    return SVGD_OK;
}

int svgd_set_timing(svgd_ctx *c, int enable)
{
    if (!c) return SVGD_ERR_ARG;
    c->timing = enable != 0;
    c->tlevel = enable < 0 ? 0 : enable;
    c->last_phi_end = nullptr;
    return SVGD_OK;
}

int svgd_get_diagnostics(svgd_ctx *c, double *out, int cap)
{
    if (!c || (!out && cap > 0)) return SVGD_ERR_ARG;
    CHK(resolve_pending(c));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->gstream) HIPCHK(c, hipStreamSynchronize(c->gstream));
    for (auto &e : c->ev_diag) {
        float ms = 0;
        HIPCHK(c, hipEventElapsedTime(&ms, e.a, e.b));
        c->dg_ms[e.kind] += ms;
        c->dg_cnt[e.kind] += 1;
        if (e.own_a) c->ev_single.push_back(e.a);
        c->ev_single.push_back(e.b);
    }
    c->ev_diag.clear();
    int ranks = 1;
    if (c->comm) (void)ncclCommCount(c->comm, &ranks);
    else if (c->hcomm) ranks = c->world;
    const double v[SVGD_DIAG_LEN] = {(double)c->h_steps,
                                     c->dg_ms[DG_PHI_KERNEL],
                                     (double)c->dg_cnt[DG_PHI_KERNEL],
                                     c->dg_ms[DG_PHI_WAIT],
                                     (double)c->dg_cnt[DG_PHI_WAIT],
                                     c->dg_ms[DG_COLL],
                                     (double)c->dg_cnt[DG_COLL],
                                     c->dg_ms[DG_GATHER_G],
                                     (double)c->dg_cnt[DG_GATHER_G],
                                     c->h_grad_ms,
                                     c->h_xwait_ms,
                                     c->h_job_ms,
                                     c->h_wait_ms,
                                     (double)ranks,
                                     (double)c->host_threads,
                                     (double)c->trk_steps,
                                     (double)c->trk_miss,
                                     (double)c->sim_world,
                                     (double)c->cpu_quota,
                                     (double)c->n_split,
                                     (double)c->n_mirror,
                                     (double)c->n_spec,
                                     c->gcomm ? 1.0 : 0.0,
                                     c->trk_band_sum};
    for (int i = 0; i < cap && i < SVGD_DIAG_LEN; ++i) out[i] = v[i];
    for (int k = 0; k < 4; ++k) c->dg_ms[k] = 0, c->dg_cnt[k] = 0;
    c->h_grad_ms = c->h_xwait_ms = c->h_job_ms = c->h_wait_ms = 0;
    c->h_steps = 0;
    c->trk_steps = c->trk_miss = 0;
    c->trk_band_sum = 0;
    c->n_split = c->n_mirror = c->n_spec = 0;
    return cap < SVGD_DIAG_LEN ? cap : SVGD_DIAG_LEN;
}

int svgd_get_timing(svgd_ctx *c, double *phi_ms, double *median_ms, int64_t *count)
{
    if (!c) return SVGD_ERR_ARG;
    CHK(resolve_pending(c));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    // the events go back to the pool: the status / scale-final marks may be
    // among them (everything they mark is complete now)
    c->ev_status_use = c->ev_fin_use = c->mark = c->phi_end = c->ev_xready_use = nullptr;
    c->last_phi_end = nullptr;
    for (auto &e : c->ev_phi) {
        float ms = 0;
        HIPCHK(c, hipEventElapsedTime(&ms, e.a, e.b));
        c->phi_ms += ms;
        c->tcount += 1;
        c->ev_pool.push_back(e.spare ? EvPair{e.spare, e.b} : EvPair{e.a, e.b});
    }
    c->ev_phi.clear();
    for (auto &e : c->ev_med) {
        float ms = 0;
        HIPCHK(c, hipEventElapsedTime(&ms, e.a, e.b));
        c->med_ms += ms;
        c->ev_pool.push_back(e.spare ? EvPair{e.spare, e.b} : EvPair{e.a, e.b});
    }
    c->ev_med.clear();
    if (phi_ms) *phi_ms = c->phi_ms;
    if (median_ms) *median_ms = c->med_ms;
    if (count) *count = c->tcount;
    c->phi_ms = c->med_ms = 0;
    c->tcount = 0;
    return SVGD_OK;
}

int svgd_phi_kernel_name(const svgd_ctx *c, char *buf, int cap)
{
    if (!c || !buf || cap <= 0) return SVGD_ERR_ARG;
    char s[96];
    const int d = c->dim;
    if (c->rowpath && c->sym) {
        std::snprintf(s, sizeof s, "k_phi_sym<%d>", d);
    } else if (c->rowpath) {
        if (c->phi_kind == 2)
            std::snprintf(s, sizeof s, "k_phi_rows<%d, %d, 8, 8192, 8>", d, c->R);
        else
            std::snprintf(s, sizeof s, "k_phi_rows<%d, %d, 4, 4096, 1>", d, c->R);
    } else if (c->dtype == SVGD_F32 && c->B3) {
        std::snprintf(s, sizeof s, "k_phi_b3<%d, %d, 8, %s, %d>", c->KP, c->NCB,
                      16 * c->NCB == d ? "true" : "false", c->b3_rg);
    } else if (c->dtype == SVGD_F32 && c->XS) {
        std::snprintf(s, sizeof s, "k_phi_f32s<%d, %d>", c->KP, c->NCB);
    } else {
        const bool f64 = c->dtype != SVGD_F32;
        int nw = 4, pre = 0;
        phi_tile_cfg(f64, &nw, &pre);
        std::snprintf(s, sizeof s, "k_phi<%s, %d, %d, %d, %s, %s>", f64 ? "double" : "float", c->KP,
                      c->NCB, nw, pre ? "true" : "false", c->dim == 16 * c->NCB ? "true" : "false");
    }
    std::snprintf(buf, (size_t)cap, "%s", s);
    return SVGD_OK;
}

int svgd_set_median_tuning(svgd_ctx *c, int64_t direct_max_pairs, int64_t sample_size,
                           int64_t candidate_capacity)
{
    if (!c) return SVGD_ERR_ARG;
    CHK(resolve_pending(c));
    if (direct_max_pairs >= 0) c->direct_max_pairs = direct_max_pairs;
    if (sample_size > 0) c->sample_size = sample_size;
    if (candidate_capacity >= 0) c->cand_capacity = candidate_capacity;
    return SVGD_OK;
}

int svgd_debug_pair_keys(svgd_ctx *c, double *out, int64_t capacity)
{
    CHK(check_ready(c));
    CHK(resolve_pending(c));
    const int64_t M = upper_pairs(c->n);
    if (capacity < M) return fail(c, SVGD_ERR_ARG, "[Argument Error] Output buffer too small.");
    if (c->world != 1)
        return fail(c, SVGD_ERR_ARG, "[Argument Error] Debug keys are single-GPU only.");
    CHK(center(c));
    double *d = nullptr;
    HIPCHK(c, hipMalloc((void **)&d, sizeof(double) * (size_t)std::max<int64_t>(1, M)));
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(c->own_tiles, 1024));
    hipError_t e = pair_pass(c, 2, grid, nullptr, 0, d);
    if (e == hipSuccess)
        e = hipMemcpyAsync(out, d, sizeof(double) * (size_t)M, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d);
    HIPCHK(c, e);
    return SVGD_OK;
}

} // extern "C"
