/*
 * svgd_oracle.c -- CPU restatement of the SVGDCpp inner step.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle and the CPU
 * baseline ("port") of bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product (svgdcpp_amd/,
 * include/) never links or calls it.
 *
 * Every function restates the reference algorithm (khaiyichin/SVGDCpp,
 * snapshot 2025-07-25, paths relative to the reference root) with the same
 * arithmetic order where the reference fixes one:
 *
 *   or_fill_eigen_random   Eigen-3.3/3.4 MatrixXd::Random with glibc rand()
 *                          (examples/{mvn,gmm}_example.cpp x0 init, tests/test_svgd.cpp:113)
 *   or_pairwise_dist_gram  GaussianRBFKernel.hpp:179-185 (Gram form XᵀX)
 *   or_median              GaussianRBFKernel.hpp:222-254 (nth_element median)
 *   or_median_scale        GaussianRBFKernel.hpp:187      a = ln(N)/med²
 *   or_phi                 SVGD.hpp:435-453 (K, Kg, (1/N)(G·K + [I..I]·Kg)),
 *                          kernel lambda GaussianRBFKernel.hpp:75-81
 *   or_adam / or_adagrad / or_rmsprop
 *                          Adam.hpp:75-96, AdaGrad.hpp:60-65, RMSProp.hpp:69-74
 *   or_apply_update        SVGD.hpp:393-399 (X += Δ, then min(upper), max(lower))
 *   or_logp_grad_gmm       MultivariateNormal.hpp:56-61 + Model.hpp:55-92,451-454
 *                          (log of an UNWEIGHTED sum of unnormalised Gaussians)
 *
 * Layout: particle matrices are d×n column-major (particle i contiguous at
 * X + i*d), exactly the reference's Eigen::MatrixXd layout (SVGD.hpp:176).
 *
 * Documented deviation: the reference takes sqrt of the Gram-form squared
 * distance, which can be slightly negative for near-coincident particles and
 * then yields NaN.  The oracle clamps it at 0.
 *
 * Pinned by: the reference's published example outputs
 * (examples/multivariate_normal/mvn_example.ipynb:3658-3668,
 *  examples/gaussian_mixture_model/gmm_example.ipynb:6396-6416) and the
 * tests/test_svgd.cpp:21-203 structural scenario -- see tests/test_oracle.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---------------------------------------------------------------- init -- */

/* Eigen 3.3/3.4 random_default_impl<double>: x + (y-x)*Scalar(rand())/RAND_MAX
 * with x=-1, y=1, evaluated in linear (column-major) order; the caller's
 * scale factor is applied afterwards (e.g. 3*Random(2,10), mvn_example.cpp:23). */
void or_fill_eigen_random(double *X, long count, double scale, unsigned seed)
{
    srand(seed);
    for (long i = 0; i < count; ++i) {
        double r = -1.0 + (2.0 * (double)rand()) / (double)RAND_MAX;
        X[i] = scale * r;
    }
}

/* splitmix64 -> uniform[-1,1): (u>>11)*2^-53*2-1 (SURVEY §8(d) synthetic inputs). */
void or_fill_splitmix(double *X, long count, double scale, uint64_t seed)
{
    uint64_t s = seed;
    for (long i = 0; i < count; ++i) {
        uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        z = z ^ (z >> 31);
        double u = (double)(z >> 11) * 0x1.0p-53;
        X[i] = scale * (u * 2.0 - 1.0);
    }
}

/* -------------------------------------------------------------- median -- */

/* GaussianRBFKernel.hpp:179-185: S = XᵀX, D² = (diag·1ᵀ + 1·diagᵀ) - 2S,
 * dist = sqrt(D²) over ALL n² entries (diagonal zeros and both triangles),
 * written column-major into out[n*n]. */
void or_pairwise_dist_gram(const double *X, int d, long n, double *out)
{
    double *diag = (double *)malloc(sizeof(double) * (size_t)n);
    for (long i = 0; i < n; ++i) {
        double s = 0.0;
        for (int k = 0; k < d; ++k) s += X[i * d + k] * X[i * d + k];
        diag[i] = s;
    }
#pragma omp parallel for schedule(static)
    for (long j = 0; j < n; ++j) {
        for (long i = 0; i < n; ++i) {
            double s = 0.0;
            for (int k = 0; k < d; ++k) s += X[i * d + k] * X[j * d + k];
            if (i == j) s = diag[i];
            double d2 = (diag[i] + diag[j]) - 2.0 * s;
            if (d2 < 0.0) d2 = 0.0; /* documented deviation (reference: NaN) */
            out[j * n + i] = sqrt(d2);
        }
    }
    free(diag);
}

static void swapd(double *a, double *b) { double t = *a; *a = *b; *b = t; }

/* nth_element: after the call v[k] holds the k-th smallest and
 * v[0..k) <= v[k] <= v[k+1..).  (Hoare-style quickselect; the values it
 * returns are the same order statistics std::nth_element returns.) */
static void nth_element_d(double *v, long n, long k)
{
    long lo = 0, hi = n - 1;
    while (hi > lo) {
        long mid = lo + (hi - lo) / 2;
        if (v[mid] < v[lo]) swapd(&v[mid], &v[lo]);
        if (v[hi] < v[lo]) swapd(&v[hi], &v[lo]);
        if (v[hi] < v[mid]) swapd(&v[hi], &v[mid]);
        double pivot = v[mid];
        long i = lo, j = hi;
        while (i <= j) {
            while (v[i] < pivot) ++i;
            while (v[j] > pivot) --j;
            if (i <= j) { swapd(&v[i], &v[j]); ++i; --j; }
        }
        if (k <= j) hi = j;
        else if (k >= i) lo = i;
        else return;
    }
}

/* GaussianRBFKernel.hpp:222-254 ComputeMedian (destroys v). */
double or_median(double *v, long count)
{
    if (count % 2 == 0) {
        long h = count / 2;
        nth_element_d(v, count, h);
        double b = v[h];
        double a = v[0];
        for (long i = 1; i < h; ++i) if (v[i] > a) a = v[i];
        return (a + b) / 2.0;
    }
    long h = count / 2;
    nth_element_d(v, count, h);
    return v[h];
}

/* GaussianRBFKernel.hpp:168-188: a = ln(n) / med², med = median of all n²
 * pairwise distances.  Returns med in *med_out, a in *a_out. */
void or_median_scale(const double *X, int d, long n, double *a_out, double *med_out)
{
    double *dist = (double *)malloc(sizeof(double) * (size_t)n * (size_t)n);
    or_pairwise_dist_gram(X, d, n, dist);
    double med = or_median(dist, n * n);
    free(dist);
    *med_out = med;
    *a_out = log((double)n) / pow(med, 2);
}

/* Exact k-th order statistic (0-based) of the upper-triangle (i<j) squared
 * distances computed in the DIRECT form sum_k (x_ik - x_jk)^2.  Used by the
 * tests to pin the GPU's selection independently of distance rounding. */
double or_upper_sqdist_kth(const double *X, int d, long n, long k)
{
    long m = n * (n - 1) / 2, p = 0;
    double *v = (double *)malloc(sizeof(double) * (size_t)(m > 0 ? m : 1));
    for (long i = 0; i < n; ++i)
        for (long j = i + 1; j < n; ++j) {
            double s = 0.0;
            for (int c = 0; c < d; ++c) {
                double t = X[i * d + c] - X[j * d + c];
                s += t * t;
            }
            v[p++] = s;
        }
    nth_element_d(v, m, k);
    double r = v[k];
    free(v);
    return r;
}

/* Rank check of a selected order statistic at sizes where the n(n-1)/2
 * distances cannot be stored: for each of nt (<= 8) thresholds t[q], the
 * number of upper-triangle (i<j) pairs whose DIRECT-form squared distance is
 * < t[q] (one streamed pass, OpenMP over rows, 64-bit counts).  s is the k-th
 * smallest iff count(< s) <= k < count(<= s); tests pass s*(1 -+ eps) to
 * absorb the last bits in which the device's centred Gram form differs. */
__attribute__((optimize("O3"))) void or_upper_sqdist_counts(const double *X, int d, long n, const double *t, int nt,
                            long long *out)
{
    long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (nt > 8) nt = 8;
    /* dimension-major copy: the j loop below is a plain vectorisable stream */
    double *Xt = (double *)malloc(sizeof(double) * (size_t)n * (size_t)d);
    for (long i = 0; i < n; ++i)
        for (int c = 0; c < d; ++c) Xt[(size_t)c * n + i] = X[(size_t)i * d + c];
    enum { JB = 512 };
#pragma omp parallel
    {
        long long loc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        double sb[JB];
#pragma omp for schedule(dynamic, 16)
        for (long i = 0; i < n; ++i) {
            for (long j0 = i + 1; j0 < n; j0 += JB) {
                const long m = (n - j0) < JB ? (n - j0) : JB;
                for (long q = 0; q < m; ++q) sb[q] = 0.0;
                for (int c = 0; c < d; ++c) {
                    const double xi = Xt[(size_t)c * n + i];
                    const double *xc = Xt + (size_t)c * n + j0;
                    for (long q = 0; q < m; ++q) {
                        const double u = xi - xc[q];
                        sb[q] += u * u;
                    }
                }
                for (int k = 0; k < nt; ++k) {
                    long long cnt = 0;
                    const double tk = t[k];
                    for (long q = 0; q < m; ++q) cnt += sb[q] < tk;
                    loc[k] += cnt;
                }
            }
        }
#pragma omp critical
        for (int k = 0; k < nt; ++k) acc[k] += loc[k];
    }
    free(Xt);
    for (int k = 0; k < nt; ++k) out[k] = acc[k];
}

/* The median work of rows [i0, i1) alone, for timing a bounded sample of a
 * large step (bench.py cpu_baseline): each row's share of the n(n-1)/2
 * distinct pairs (partners i+1 .. i+floor(n/2), cyclic), Gram-form distances
 * as GaussianRBFKernel.hpp:179-185, then the nth_element of
 * ComputeMedian (:222-254) over those values.  Returns the sample median. */
double or_median_rows_work(const double *X, int d, long n, long i0, long i1)
{
    const long h = n / 2, rows = i1 - i0;
    double *diag = (double *)malloc(sizeof(double) * (size_t)n);
    double *v = (double *)malloc(sizeof(double) * (size_t)(rows * h > 0 ? rows * h : 1));
#pragma omp parallel for schedule(static)
    for (long i = 0; i < n; ++i) {
        double s = 0.0;
        for (int k = 0; k < d; ++k) s += X[i * d + k] * X[i * d + k];
        diag[i] = s;
    }
#pragma omp parallel for schedule(static)
    for (long r = 0; r < rows; ++r) {
        const long i = i0 + r;
        for (long q = 1; q <= h; ++q) {
            const long j = (i + q) % n;
            double s = 0.0;
            for (int k = 0; k < d; ++k) s += X[i * d + k] * X[j * d + k];
            double d2 = (diag[i] + diag[j]) - 2.0 * s;
            v[r * h + (q - 1)] = sqrt(d2 < 0.0 ? 0.0 : d2);
        }
    }
    double med = rows * h > 0 ? or_median(v, rows * h) : 0.0;
    free(v);
    free(diag);
    return med;
}

/* ----------------------------------------------------------------- phi -- */

/* SVGD.hpp:435-453 with the RBF lambda GaussianRBFKernel.hpp:75-81 and
 * M = a·I:
 *   K[j,i]          = exp( (-diff)ᵀ M diff ),   diff = x_j - x_i
 *   Kg[j*d+k, i]    = -2 a diff_k K[j,i]        (∂/∂x_j, location x_i)
 *   phi[:, i]       = (1/N) (Σ_j G[:,j] K[j,i] + Σ_j Kg[j*d:(j+1)*d, i])
 * Rows i in [i0, i1) are computed (pass 0, n for all).  K (n×n) and Kg
 * (dn×n) are materialised column-major when non-NULL (full range only).
 * M is applied as in the reference product: r_k = Σ_l (-diff_l) M_lk with
 * M diagonal, i.e. r_k = -(diff_k) * a, then u = Σ_k r_k diff_k. */
void or_phi_rows(const double *X, const double *G, int d, long n, double a,
                 long i0, long i1, double *phi, double *K, double *Kg)
{
    const double inv_n = 1.0 / (double)n;
#pragma omp parallel for schedule(dynamic, 16)
    for (long i = i0; i < i1; ++i) {
        double accg[256], acck[256];
        double *diff = (double *)malloc(sizeof(double) * (size_t)d);
        for (int k = 0; k < d; ++k) { accg[k] = 0.0; acck[k] = 0.0; }
        const double *xi = X + i * d;
        for (long j = 0; j < n; ++j) {
            const double *xj = X + j * d;
            double u = 0.0;
            for (int k = 0; k < d; ++k) diff[k] = xj[k] - xi[k];
            for (int k = 0; k < d; ++k) u += (-diff[k] * a) * diff[k];
            double kv = exp(u);
            if (K) K[i * n + j] = kv;
            for (int k = 0; k < d; ++k) {
                double g = -2.0 * a * diff[k] * kv;
                if (Kg) Kg[i * (n * (long)d) + j * d + k] = g;
                accg[k] += G[j * d + k] * kv;
                acck[k] += g;
            }
        }
        for (int k = 0; k < d; ++k) phi[(i - i0) * d + k] = inv_n * (accg[k] + acck[k]);
        free(diff);
    }
}

void or_phi(const double *X, const double *G, int d, long n, double a,
            double *phi, double *K, double *Kg)
{
    or_phi_rows(X, G, d, n, a, 0, n, phi, K, Kg);
}

/* ----------------------------------------------------------- optimizers -- */

/* Adam.hpp:75-83 (+ CorrectForBias :93-96).  t is the counter AFTER the
 * increment (the reference increments before use). */
void or_adam(double *m, double *v, const double *g, long cnt, long t,
             double lr, double b1, double b2, double eps, double *delta)
{
    double c1 = 1.0 - pow(b1, (double)t), c2 = 1.0 - pow(b2, (double)t);
    for (long e = 0; e < cnt; ++e) {
        m[e] = b1 * m[e] + (1 - b1) * g[e];
        v[e] = b2 * v[e] + (1 - b2) * (g[e] * g[e]);
    }
    for (long e = 0; e < cnt; ++e)
        delta[e] = (lr * (1.0 / (eps + sqrt(v[e] / c2)))) * (m[e] / c1);
}

/* AdaGrad.hpp:60-65 */
void or_adagrad(double *v, const double *g, long cnt, double lr, double eps, double *delta)
{
    for (long e = 0; e < cnt; ++e) v[e] += g[e] * g[e];
    for (long e = 0; e < cnt; ++e) delta[e] = (lr * (1.0 / (eps + sqrt(v[e])))) * g[e];
}

/* RMSProp.hpp:69-74 */
void or_rmsprop(double *v, const double *g, long cnt, double lr, double beta,
                double eps, double *delta)
{
    for (long e = 0; e < cnt; ++e) v[e] = beta * v[e] + (1 - beta) * (g[e] * g[e]);
    for (long e = 0; e < cnt; ++e) delta[e] = (lr * (1.0 / (eps + sqrt(v[e])))) * g[e];
}

/* SVGD.hpp:393-399: X += Δ; if bounded X = max(min(X, upper), lower) with
 * d-vector bounds replicated over particles (NULL = unbounded). */
void or_apply_update(double *X, const double *delta, int d, long n,
                     const double *lower, const double *upper)
{
    for (long i = 0; i < n; ++i)
        for (int k = 0; k < d; ++k) {
            double x = X[i * d + k] + delta[i * d + k];
            if (lower && upper) {
                x = x < upper[k] ? x : upper[k];
                x = x > lower[k] ? x : lower[k];
            }
            X[i * d + k] = x;
        }
}

/* ---------------------------------------------------------------- model -- */

/* In-place Gauss-Jordan inverse with partial pivoting (row-major d×d). */
static void invert(double *A, int d, double *out)
{
    double *M = (double *)malloc(sizeof(double) * (size_t)d * d * 2);
    for (int r = 0; r < d; ++r)
        for (int c = 0; c < 2 * d; ++c)
            M[r * 2 * d + c] = c < d ? A[r * d + c] : (c - d == r ? 1.0 : 0.0);
    for (int c = 0; c < d; ++c) {
        int p = c;
        for (int r = c + 1; r < d; ++r)
            if (fabs(M[r * 2 * d + c]) > fabs(M[p * 2 * d + c])) p = r;
        if (p != c)
            for (int q = 0; q < 2 * d; ++q) swapd(&M[c * 2 * d + q], &M[p * 2 * d + q]);
        double piv = M[c * 2 * d + c];
        for (int q = 0; q < 2 * d; ++q) M[c * 2 * d + q] /= piv;
        for (int r = 0; r < d; ++r) {
            if (r == c) continue;
            double f = M[r * 2 * d + c];
            for (int q = 0; q < 2 * d; ++q) M[r * 2 * d + q] -= f * M[c * 2 * d + q];
        }
    }
    for (int r = 0; r < d; ++r)
        for (int c = 0; c < d; ++c) out[r * d + c] = M[r * 2 * d + d + c];
    free(M);
}

/* ∇ log Σ_c exp(-½ (x-μ_c)ᵀ Σ_c⁻¹ (x-μ_c)) for n particles (k components;
 * k = 1 is MultivariateNormal.hpp:56-61 alone).  mu: k×d, cov: k×d×d
 * (symmetric).  Written with a max-shift (log-sum-exp); SURVEY Appendix A.7. */
void or_logp_grad_gmm(const double *X, int d, long n, int k, const double *mu,
                      const double *cov, double *G)
{
    double *prec = (double *)malloc(sizeof(double) * (size_t)k * d * d);
    for (int c = 0; c < k; ++c) invert((double *)cov + (size_t)c * d * d, d, prec + (size_t)c * d * d);
#pragma omp parallel for schedule(static)
    for (long i = 0; i < n; ++i) {
        double q[64], gc[64 * 64], diff[256];
        const double *x = X + i * d;
        double qmin = INFINITY;
        for (int c = 0; c < k; ++c) {
            const double *P = prec + (size_t)c * d * d;
            for (int r = 0; r < d; ++r) diff[r] = x[r] - mu[c * d + r];
            double qq = 0.0;
            for (int r = 0; r < d; ++r) {
                double s = 0.0;
                for (int l = 0; l < d; ++l) s += P[r * d + l] * diff[l];
                gc[c * d + r] = -s;
                qq += diff[r] * s;
            }
            q[c] = 0.5 * qq;
            if (q[c] < qmin) qmin = q[c];
        }
        double wsum = 0.0;
        for (int c = 0; c < k; ++c) { q[c] = exp(-(q[c] - qmin)); wsum += q[c]; }
        for (int r = 0; r < d; ++r) {
            double s = 0.0;
            for (int c = 0; c < k; ++c) s += q[c] * gc[c * d + r];
            G[i * d + r] = s / wsum;
        }
    }
    free(prec);
}

/* -∑_i ∇² log p(x_i) for the Gaussian-sum model over n particles, the sum
 * inside the Hessian scale (GaussianRBFKernel.hpp:189-210 with
 * Model::EvaluateLogModelHessian, Model.hpp:366-370).  With w = softmax(-q/2)
 * and g_c = -P_c (x - μ_c):
 *   ∇² log p = ∑_c w_c (g_c g_cᵀ - P_c) - (∑_c w_c g_c)(∑_c w_c g_c)ᵀ.
 * H_out: d×d row-major (symmetric), accumulated serially in particle order. */
void or_neg_hess_sum_gmm(const double *X, int d, long n, int k, const double *mu,
                         const double *cov, double *H_out)
{
    double *prec = (double *)malloc(sizeof(double) * (size_t)k * d * d);
    for (int c = 0; c < k; ++c) invert((double *)cov + (size_t)c * d * d, d, prec + (size_t)c * d * d);
    double *H = (double *)calloc((size_t)d * d, sizeof(double));
    double q[64], gc[64 * 64], diff[256], gbar[256];
    for (long i = 0; i < n; ++i) {
        const double *x = X + i * d;
        double qmin = INFINITY;
        for (int c = 0; c < k; ++c) {
            const double *P = prec + (size_t)c * d * d;
            for (int r = 0; r < d; ++r) diff[r] = x[r] - mu[c * d + r];
            double qq = 0.0;
            for (int r = 0; r < d; ++r) {
                double s = 0.0;
                for (int l = 0; l < d; ++l) s += P[r * d + l] * diff[l];
                gc[c * d + r] = -s;
                qq += diff[r] * s;
            }
            q[c] = 0.5 * qq;
            if (q[c] < qmin) qmin = q[c];
        }
        double wsum = 0.0;
        for (int c = 0; c < k; ++c) { q[c] = exp(-(q[c] - qmin)); wsum += q[c]; }
        for (int c = 0; c < k; ++c) q[c] /= wsum;
        for (int r = 0; r < d; ++r) {
            double s = 0.0;
            for (int c = 0; c < k; ++c) s += q[c] * gc[c * d + r];
            gbar[r] = s;
        }
        for (int r = 0; r < d; ++r)
            for (int l = 0; l < d; ++l) {
                double h = 0.0;
                for (int c = 0; c < k; ++c)
                    h += q[c] * (gc[c * d + r] * gc[c * d + l] - prec[(size_t)c * d * d + r * d + l]);
                h -= gbar[r] * gbar[l];
                H[r * d + l] -= h;
            }
    }
    memcpy(H_out, H, sizeof(double) * (size_t)d * d);
    free(H);
    free(prec);
}

/* φ̂ for a full (symmetric) kernel scale matrix M: k(x, x') = exp(-(x-x')ᵀ M (x-x')),
 * ∇ₓ k = -2 M (x - x') k (GaussianRBFKernel.hpp:75-81 with M = kernel_parameters_[0],
 * the Hessian scale of :189-210 or a user-set constant).  Rows [i0, i1). */
void or_phi_matrix_rows(const double *X, const double *G, int d, long n, const double *M,
                        long i0, long i1, double *phi)
{
    const double inv_n = 1.0 / (double)n;
#pragma omp parallel for schedule(dynamic, 16)
    for (long i = i0; i < i1; ++i) {
        double accg[256], acck[256], diff[256], Md[256];
        for (int k = 0; k < d; ++k) { accg[k] = 0.0; acck[k] = 0.0; }
        const double *xi = X + i * d;
        for (long j = 0; j < n; ++j) {
            const double *xj = X + j * d;
            for (int k = 0; k < d; ++k) diff[k] = xj[k] - xi[k];
            double u = 0.0;
            for (int r = 0; r < d; ++r) {
                double s = 0.0;
                for (int l = 0; l < d; ++l) s += M[r * d + l] * diff[l];
                Md[r] = s;
                u += diff[r] * s;
            }
            const double kv = exp(-u);
            for (int k = 0; k < d; ++k) {
                accg[k] += G[j * d + k] * kv;
                acck[k] += -2.0 * Md[k] * kv;
            }
        }
        for (int k = 0; k < d; ++k) phi[(i - i0) * d + k] = inv_n * (accg[k] + acck[k]);
    }
}

int or_num_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* thread count of the OpenMP loops (the cpu_baseline's 1-thread run) */
void or_set_threads(int n)
{
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}
