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

// Rows [i0, i0 + np) (np <= 4), cloned for AVX2 + FMA hosts (a
// runtime-dispatched ifunc; the generic clone runs elsewhere; called per block
// because an OpenMP region's outlined body would not inherit the clone's
// target).  For each 8-wide slice of r the 4 x 8 sums stay in registers while
// l runs (one load of the precision row feeds 4 particles); every
// s_r = sum_l P[r][l] diff[l] is still accumulated from 0 with l ascending.
constexpr int GB_NP = 4, GB_RW = 8;
typedef double v4d __attribute__((vector_size(32)));
__attribute__((target_clones("arch=haswell", "default"))) static void
logp_grad_block(const HostModel *m, const double *X, int64_t i0, int np, double *G, double *diff,
                double *gc, double *q)
{
    const int d = m->d, k = m->k;
    for (int c = 0; c < k; ++c) {
        const double *PT = m->precT.data() + (size_t)c * d * d;
        const double *mu = m->mu.data() + (size_t)c * d;
        for (int p = 0; p < GB_NP; ++p)
            for (int r = 0; r < d; ++r)
                diff[(size_t)p * d + r] = p < np ? X[(i0 + p) * d + r] - mu[r] : 0.0;
        int r0 = 0;
        for (; r0 + GB_RW <= d; r0 += GB_RW) {
            v4d acc[GB_NP][2] = {};
            for (int l = 0; l < d; ++l) {
                const double *row = PT + (size_t)l * d + r0;
                v4d a0, a1;
                std::memcpy(&a0, row, sizeof a0);
                std::memcpy(&a1, row + 4, sizeof a1);
                for (int p = 0; p < GB_NP; ++p) {
                    const double dl = diff[(size_t)p * d + l];
                    const v4d b = {dl, dl, dl, dl};
                    acc[p][0] += a0 * b;
                    acc[p][1] += a1 * b;
                }
            }
            for (int p = 0; p < GB_NP; ++p)
                std::memcpy(gc + ((size_t)p * k + c) * d + r0, acc[p], sizeof acc[p]);
        }
        for (int p = 0; p < GB_NP; ++p)
            for (int r = r0; r < d; ++r) {
                double sr = 0.0;
                for (int l = 0; l < d; ++l) sr += PT[(size_t)l * d + r] * diff[(size_t)p * d + l];
                gc[((size_t)p * k + c) * d + r] = sr;
            }
        for (int p = 0; p < GB_NP; ++p) {
            double *sp = gc + ((size_t)p * k + c) * d;
            double qq = 0.0;
            for (int r = 0; r < d; ++r) {
                qq += diff[(size_t)p * d + r] * sp[r];
                sp[r] = -sp[r];
            }
            q[(size_t)p * k + c] = 0.5 * qq;
        }
    }
    for (int p = 0; p < np; ++p) {
        double *qp = q + (size_t)p * k;
        double qmin = INFINITY;
        for (int c = 0; c < k; ++c) qmin = qp[c] < qmin ? qp[c] : qmin;
        double wsum = 0.0;
        for (int c = 0; c < k; ++c) {
            qp[c] = std::exp(-(qp[c] - qmin));
            wsum += qp[c];
        }
        const double *gp = gc + (size_t)p * k * d;
        for (int r = 0; r < d; ++r) {
            double sr = 0.0;
            for (int c = 0; c < k; ++c) sr += qp[c] * gp[(size_t)c * d + r];
            G[(i0 + p) * d + r] = sr / wsum;
        }
    }
}

static void logp_grad_rows(const HostModel *m, const double *X, int64_t nrows, double *G)
{
    const int d = m->d, k = m->k;
#pragma omp parallel
    {
        std::vector<double> diff((size_t)GB_NP * d), gc((size_t)GB_NP * k * d), q((size_t)GB_NP * k);
        const int64_t nblk = (nrows + GB_NP - 1) / GB_NP;
#pragma omp for schedule(static)
        for (int64_t b = 0; b < nblk; ++b) {
            const int64_t i0 = b * GB_NP;
            logp_grad_block(m, X, i0, (int)std::min<int64_t>(GB_NP, nrows - i0), G, diff.data(),
                            gc.data(), q.data());
        }
    }
}

int svgd_model_logp_grad(void *model, const double *X, int64_t nrows, double *G)
{
    const HostModel *m = static_cast<const HostModel *>(model);
    if (!m || (!X && nrows > 0) || (!G && nrows > 0)) return SVGD_ERR_ARG;
    logp_grad_rows(m, X, nrows, G);
    return SVGD_OK;
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
