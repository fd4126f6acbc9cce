// host_models.cpp -- built-in target models, evaluated on the host.
//
// The reference keeps ∇log p on the host (Model::EvaluateLogModelGrad,
// include/SVGDCpp/Model/Model.hpp:335-338) and so does this build: the
// device step receives G = ∇log p(X_t) once per step.  CppAD is not
// available, so the built-in models use their closed forms (the "override
// EvaluateLogModelGrad" route of the reference's doc/instructions.md:234-301):
//
//   MultivariateNormal  p(x) = exp(-½ (x-μ)ᵀ Σ⁻¹ (x-μ))     MultivariateNormal.hpp:56-61
//                       ∇log p = -Σ⁻¹ (x-μ)
//   mvn_1 + ... + mvn_k log Σ_c exp(-½ q_c(x)), unweighted and unnormalised,
//                       the reference's Model::operator+ (Model.hpp:55-92)
//                       ∇log p = Σ_c w_c (-Σ_c⁻¹ (x-μ_c)),  w = softmax(-½ q)
//
// Rows are evaluated in parallel with OpenMP (the reference evaluates them
// serially even in parallel mode, SVGD.hpp:412-416).
#include <algorithm>
#include <cmath>
#include <omp.h>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/svgdcpp_amd/svgd_capi.h"
#include "host_models.h"

using svgd_amd::HostModel;

namespace {

// Gauss-Jordan inverse with partial pivoting; false if singular.
bool invert(const double *A, int d, double *out)
{
    std::vector<double> M((size_t)d * 2 * d);
    for (int r = 0; r < d; ++r)
        for (int c = 0; c < 2 * d; ++c)
            M[(size_t)r * 2 * d + c] = c < d ? A[r * d + c] : (c - d == r ? 1.0 : 0.0);
    for (int c = 0; c < d; ++c) {
        int p = c;
        for (int r = c + 1; r < d; ++r)
            if (std::fabs(M[(size_t)r * 2 * d + c]) > std::fabs(M[(size_t)p * 2 * d + c])) p = r;
        if (M[(size_t)p * 2 * d + c] == 0.0) return false;
        if (p != c)
            for (int q = 0; q < 2 * d; ++q) std::swap(M[(size_t)c * 2 * d + q], M[(size_t)p * 2 * d + q]);
        const double piv = M[(size_t)c * 2 * d + c];
        for (int q = 0; q < 2 * d; ++q) M[(size_t)c * 2 * d + q] /= piv;
        for (int r = 0; r < d; ++r) {
            if (r == c) continue;
            const double f = M[(size_t)r * 2 * d + c];
            if (f == 0.0) continue;
            for (int q = 0; q < 2 * d; ++q) M[(size_t)r * 2 * d + q] -= f * M[(size_t)c * 2 * d + q];
        }
    }
    for (int r = 0; r < d; ++r)
        for (int c = 0; c < d; ++c) out[r * d + c] = M[(size_t)r * 2 * d + d + c];
    return true;
}

} // namespace

// Rows [i0, i0 + np) (np <= 4), two builds of one body (host_grad_block.inc):
// the baseline x86-64 one and an AVX2 + FMA one, chosen once at run time by
// the CPU's features (GCC's target_clones keys "arch=" clones on the CPU
// model, so an AMD host never got its AVX2 clone: 46.7 vs 11.3 ms single
// thread at N = 65536, d = 64).  For each 8-wide slice of r the 4 x 8 sums
// stay in registers while l runs (one load of the precision row feeds 4
// particles); every s_r = sum_l P[r][l] diff[l] is accumulated from 0 with
// l ascending, whatever the blocking.
constexpr int GB_NP = 4, GB_RW = 8;
typedef double v4d __attribute__((vector_size(32)));
namespace gb_base { // (-Wno-psabi: exp4_nonpos's v4d return is inlined, no ABI crossing)
#include "host_grad_block.inc"
}
#pragma GCC push_options
#pragma GCC target("avx2,fma")
namespace gb_avx2 {
#include "host_grad_block.inc"
}
#pragma GCC pop_options

// AVX-512 hosts (the MI355X boxes' EPYC 9575F): 8 particles per call, one
// per vector lane (host_grad_soa8.inc) -- about a quarter of the AVX2
// block's instructions at d = 8, k = 4
#pragma GCC push_options
#pragma GCC target("avx512f,avx512dq,fma")
namespace gb_avx512 {
#include "host_grad_soa8.inc"
}
#pragma GCC pop_options

typedef void (*GradBlockFn)(const HostModel *, const double *, int64_t, int, double *, double *, double *,
                            double *);
GradBlockFn pick_grad_block()
{
    __builtin_cpu_init();
    return (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma")) ? gb_avx2::logp_grad_block
                                                                           : gb_base::logp_grad_block;
}
bool have_avx512()
{
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq") &&
           __builtin_cpu_supports("fma");
}

// variant: 0 the host's best, 1 the 4-particle block (AVX2 / baseline), 2 SoA8 (AVX-512).
// Returns SVGD_ERR_RUNTIME when a thread's work area cannot be allocated.
static int logp_grad_rows(const HostModel *m, const double *X, int64_t nrows, double *G,
                           int nthreads, int variant = 0)
{
    static const GradBlockFn block = pick_grad_block();
    static const bool avx512 = have_avx512();
    const int d = m->d, k = m->k;
    if (nthreads <= 0) nthreads = omp_get_max_threads();
    const bool soa8 = variant == 2 || (variant == 0 && avx512);
    if (soa8 && !avx512) return SVGD_ERR_ARG; // (variant 2 forced on a host without AVX-512: refused by the caller)
    int failed = 0;
#pragma omp parallel num_threads(nthreads)
    {
        if (soa8) {
            // 64-byte aligned by hand: outside the AVX-512 target a 64-byte
            // vector type is not 64-byte aligned by the allocator
            const size_t bytes = sizeof(double) * 8 * ((size_t)(2 + k) * d + k);
            double *ws = static_cast<double *>(std::aligned_alloc(64, (bytes + 63) / 64 * 64));
            if (!ws) {
#pragma omp atomic write
                failed = 1;
            }
            const int64_t nblk = (nrows + 7) / 8;
            // (every thread reaches the worksharing loop; one without its
            // work area skips its blocks and the call reports the failure)
#pragma omp for schedule(static)
            for (int64_t b = 0; b < nblk; ++b)
                if (ws) gb_avx512::logp_grad_soa8(m, X, b * 8, (int)std::min<int64_t>(8, nrows - b * 8), G, ws);
            std::free(ws);
        } else {
            std::vector<double> diff((size_t)GB_NP * d), gc((size_t)GB_NP * k * d), q((size_t)GB_NP * k);
            const int64_t nblk = (nrows + GB_NP - 1) / GB_NP;
#pragma omp for schedule(static)
            for (int64_t b = 0; b < nblk; ++b) {
                const int64_t i0 = b * GB_NP;
                block(m, X, i0, (int)std::min<int64_t>(GB_NP, nrows - i0), G, diff.data(), gc.data(),
                      q.data());
            }
        }
    }
    return failed ? SVGD_ERR_RUNTIME : SVGD_OK;
}

namespace svgd_amd {
int model_logp_grad_threads(const HostModel *m, const double *X, int64_t nrows, double *G,
                            int nthreads)
{
    if (!m || (!X && nrows > 0) || (!G && nrows > 0)) return SVGD_ERR_ARG;
    return logp_grad_rows(m, X, nrows, G, nthreads);
}
bool host_grad_avx512() { return have_avx512(); }
int model_logp_grad_variant(const HostModel *m, const double *X, int64_t nrows, double *G, int nthreads,
                            int variant)
{
    if (!m || (!X && nrows > 0) || (!G && nrows > 0) || variant < 0 || variant > 2) return SVGD_ERR_ARG;
    if (variant == 2 && !have_avx512()) return SVGD_ERR_ARG;
    return logp_grad_rows(m, X, nrows, G, nthreads, variant);
}
} // namespace svgd_amd

extern "C" {

int svgd_model_create(void **out, int dim, int ncomp, const double *mus, const double *covs)
{
    if (!out || dim <= 0 || ncomp <= 0 || !mus || !covs) return SVGD_ERR_ARG;
    HostModel *m = new (std::nothrow) HostModel();
    if (!m) return SVGD_ERR_RUNTIME;
    m->d = dim;
    m->k = ncomp;
    m->mu.assign(mus, mus + (size_t)ncomp * dim);
    m->prec.resize((size_t)ncomp * dim * dim);
    for (int c = 0; c < ncomp; ++c)
        if (!invert(covs + (size_t)c * dim * dim, dim, m->prec.data() + (size_t)c * dim * dim)) {
            delete m;
            return SVGD_ERR_ARG;
        }
    m->precT.resize(m->prec.size());
    for (int c = 0; c < ncomp; ++c)
        for (int r = 0; r < dim; ++r)
            for (int l = 0; l < dim; ++l)
                m->precT[((size_t)c * dim + l) * dim + r] = m->prec[((size_t)c * dim + r) * dim + l];
    *out = m;
    return SVGD_OK;
}

int svgd_model_destroy(void *model)
{
    delete static_cast<HostModel *>(model);
    return SVGD_OK;
}

int svgd_model_logp_grad(void *model, const double *X, int64_t nrows, double *G)
{
    const HostModel *m = static_cast<const HostModel *>(model);
    if (!m || (!X && nrows > 0) || (!G && nrows > 0)) return SVGD_ERR_ARG;
    return logp_grad_rows(m, X, nrows, G, 0);
}

int svgd_model_neg_hess_sum(void *model, const double *X, int64_t nrows, double *H)
{
    // -sum_i hess log p(x_i) (GaussianRBFKernel.hpp:197-205 with
    // Model::EvaluateLogModelHessian, Model.hpp:366-370), closed form:
    //   hess log p = sum_c w_c (g_c g_c^T - P_c) - gbar gbar^T,  gbar = sum_c w_c g_c,
    // w = softmax(-q/2), g_c = -P_c (x - mu_c).  Per-thread partial sums are
    // added in thread order (deterministic for a fixed thread count).
    const HostModel *m = static_cast<const HostModel *>(model);
    if (!m || !H || (!X && nrows > 0)) return SVGD_ERR_ARG;
    const int d = m->d, k = m->k;
    const size_t dd = (size_t)d * d;
    std::vector<std::vector<double>> part;
#pragma omp parallel
    {
#pragma omp single
        part.assign((size_t)omp_get_num_threads(), std::vector<double>(dd, 0.0));
        std::vector<double> &Hp = part[(size_t)omp_get_thread_num()];
        std::vector<double> diff(d), gc((size_t)k * d), q(k), gbar(d);
#pragma omp for schedule(static)
        for (int64_t i = 0; i < nrows; ++i) {
            const double *x = X + i * d;
            double qmin = INFINITY;
            for (int c = 0; c < k; ++c) {
                const double *P = m->prec.data() + (size_t)c * dd;
                const double *mu = m->mu.data() + (size_t)c * d;
                for (int r = 0; r < d; ++r) diff[r] = x[r] - mu[r];
                double qq = 0.0;
                for (int r = 0; r < d; ++r) {
                    double s = 0.0;
                    for (int l = 0; l < d; ++l) s += P[r * d + l] * diff[l];
                    gc[(size_t)c * d + r] = -s;
                    qq += diff[r] * s;
                }
                q[c] = 0.5 * qq;
                qmin = q[c] < qmin ? q[c] : qmin;
            }
            double wsum = 0.0;
            for (int c = 0; c < k; ++c) {
                q[c] = std::exp(-(q[c] - qmin));
                wsum += q[c];
            }
            for (int c = 0; c < k; ++c) q[c] /= wsum;
            for (int r = 0; r < d; ++r) {
                double s = 0.0;
                for (int c = 0; c < k; ++c) s += q[c] * gc[(size_t)c * d + r];
                gbar[r] = s;
            }
            for (int r = 0; r < d; ++r)
                for (int l = 0; l < d; ++l) {
                    double h = 0.0;
                    for (int c = 0; c < k; ++c)
                        h += q[c] * (gc[(size_t)c * d + r] * gc[(size_t)c * d + l] -
                                     m->prec[(size_t)c * dd + (size_t)r * d + l]);
                    Hp[(size_t)r * d + l] -= h - gbar[r] * gbar[l];
                }
        }
    }
    for (size_t e = 0; e < dd; ++e) H[e] = 0.0;
    for (const auto &Hp : part)
        for (size_t e = 0; e < dd; ++e) H[e] += Hp[e];
    return SVGD_OK;
}

} // extern "C"
