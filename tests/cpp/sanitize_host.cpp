// Host-code sanitizer driver (AddressSanitizer + UndefinedBehaviorSanitizer):
// the planner (plan.cpp), the host Gaussian-sum models (host_models.cpp) and
// the CPU oracle (oracle/svgd_oracle.c, test infrastructure) built with
// -fsanitize=address,undefined and exercised with cross-checks
// (`make sanitize`, run by tests/test_sanitize.py).  The HIP-side host code
// (svgd_capi.cpp, hostcomm.cpp) drives the GPU and is covered by the -m gpu
// tests instead: GPU sanitizers are not available on this pool.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/svgdcpp_amd/svgd_capi.h"

extern "C" {
void or_fill_splitmix(double *X, long count, double scale, uint64_t seed);
void or_median_scale(const double *X, int d, long n, double *a_out, double *med_out);
double or_upper_sqdist_kth(const double *X, int d, long n, long k);
void or_phi_rows(const double *X, const double *G, int d, long n, double a, long i0, long i1,
                 double *phi, double *K, double *Kg);
void or_logp_grad_gmm(const double *X, int d, long n, int k, const double *mu,
                      const double *covs, double *G);
void or_neg_hess_sum_gmm(const double *X, int d, long n, int k, const double *mu,
                         const double *covs, double *H);
void or_phi_matrix_rows(const double *X, const double *G, int d, long n, const double *M,
                        long i0, long i1, double *out);
}

static int failures = 0;
#define CHECK(cond)                                                                           \
    do {                                                                                      \
        if (!(cond)) {                                                                        \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond);      \
            ++failures;                                                                       \
        }                                                                                     \
    } while (0)

static void test_plan()
{
    // row shards tile [0, n) exactly
    for (int64_t n : {1, 2, 7, 64, 1000, 65537})
        for (int world : {1, 2, 3, 8}) {
            int64_t next = 0;
            for (int r = 0; r < world; ++r) {
                int64_t a, b;
                svgd_plan_rows(n, world, r, &a, &b);
                CHECK(a == next && b >= a && b <= n);
                next = b;
            }
            CHECK(next == n);
        }
    // median ranks of the n^2 list
    for (int64_t n : {1, 2, 3, 4, 5, 100, 101}) {
        int64_t lo, hi;
        const int navg = svgd_plan_median_ranks(n, &lo, &hi);
        CHECK(navg == 1 || navg == 2);
        CHECK(lo <= hi);
    }
    // pair tiles: every unordered block pair exactly once over the ranks
    for (int64_t n : {5, 300, 1000})
        for (int block : {64, 256})
            for (int world : {1, 2, 3}) {
                const int64_t nb = (n + block - 1) / block;
                std::vector<int> seen(nb * nb, 0);
                int64_t tot = 0;
                for (int r = 0; r < world; ++r) {
                    const int64_t t = svgd_plan_pair_tiles(n, block, world, r);
                    tot += t;
                    for (int64_t k = 0; k < t; ++k) {
                        int64_t I, J;
                        svgd_plan_pair_tile(n, block, world, r, k, &I, &J);
                        CHECK(I >= 0 && I < nb && J >= 0 && J < nb);
                        const int64_t a = I < J ? I : J, b = I < J ? J : I;
                        seen[a * nb + b] += 1;
                    }
                }
                CHECK(tot == nb * (nb + 1) / 2);
                for (int64_t a = 0; a < nb; ++a)
                    for (int64_t b = a; b < nb; ++b) CHECK(seen[a * nb + b] == 1);
            }
    // bucket select against a direct scan
    std::vector<unsigned long long> cnt(2048);
    uint64_t s = 12345;
    for (auto &c : cnt) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        c = (s >> 33) % 7;
    }
    int64_t total = 0;
    for (auto c : cnt) total += (int64_t)c;
    for (int64_t r0 : {int64_t(0), total / 3, total - 1}) {
        const int64_t ranks[2] = {r0, r0 + (r0 + 1 < total ? 1 : 0)};
        int bsel[2];
        int64_t rin[2], tot = 0;
        CHECK(svgd_plan_bucket_select(cnt.data(), 2048, 2, ranks, bsel, rin, &tot) == 0);
        for (int q = 0; q < 2; ++q) {
            int64_t cum = 0;
            for (int b = 0; b < bsel[q]; ++b) cum += (int64_t)cnt[b];
            CHECK(cum + rin[q] == ranks[q] && rin[q] < (int64_t)cnt[bsel[q]]);
        }
    }
    const int64_t bad[2] = {total, total};
    int bsel[2];
    int64_t rin[2], tot = 0;
    CHECK(svgd_plan_bucket_select(cnt.data(), 2048, 2, bad, bsel, rin, &tot) == -1);
}

static void test_models_vs_oracle()
{
    const int d = 5, k = 3;
    const long n = 257;
    std::vector<double> X(n * d), mu(k * d), cov(k * d * d, 0.0);
    or_fill_splitmix(X.data(), n * d, 3.0, 0x5EED);
    or_fill_splitmix(mu.data(), k * d, 2.0, 0x5EEE);
    for (int c = 0; c < k; ++c)
        for (int r = 0; r < d; ++r) {
            cov[(c * d + r) * d + r] = 1.0 + 0.25 * c;
            if (r + 1 < d) cov[(c * d + r) * d + r + 1] = cov[(c * d + r + 1) * d + r] = 0.1;
        }
    void *m = nullptr;
    CHECK(svgd_model_create(&m, d, k, mu.data(), cov.data()) == SVGD_OK);
    std::vector<double> G(n * d), Gr(n * d), H(d * d), Hr(d * d);
    CHECK(svgd_model_logp_grad(m, X.data(), n, G.data()) == SVGD_OK);
    or_logp_grad_gmm(X.data(), d, n, k, mu.data(), cov.data(), Gr.data());
    double err = 0;
    for (long e = 0; e < n * d; ++e) err = std::fmax(err, std::fabs(G[e] - Gr[e]));
    CHECK(err <= 1e-12);
    CHECK(svgd_model_neg_hess_sum(m, X.data(), n, H.data()) == SVGD_OK);
    or_neg_hess_sum_gmm(X.data(), d, n, k, mu.data(), cov.data(), Hr.data());
    err = 0;
    for (int e = 0; e < d * d; ++e) err = std::fmax(err, std::fabs(H[e] - Hr[e]) / (1 + std::fabs(Hr[e])));
    CHECK(err <= 1e-10);
    CHECK(svgd_model_destroy(m) == SVGD_OK);
    m = nullptr;
    CHECK(svgd_model_create(&m, d, k, mu.data(), nullptr) == SVGD_ERR_ARG && m == nullptr);
}

static void test_oracle_paths()
{
    const int d = 3;
    const long n = 97;
    std::vector<double> X(n * d), G(n * d), ph(n * d), pm(n * d);
    or_fill_splitmix(X.data(), n * d, 1.0, 7);
    or_fill_splitmix(G.data(), n * d, 1.0, 8);
    double a = 0, med = 0;
    or_median_scale(X.data(), d, n, &a, &med);
    CHECK(med > 0 && std::isfinite(a));
    // the median of the n^2 list is the mean of two upper-list order statistics here
    const double lo = or_upper_sqdist_kth(X.data(), d, n, 0);
    CHECK(lo >= 0);
    std::vector<double> K(n * n), Kg(n * n * d);
    or_phi_rows(X.data(), G.data(), d, n, a, 0, n, ph.data(), K.data(), Kg.data());
    CHECK(K[0] == 1.0); // the diagonal
    // the matrix form with M = a I equals the isotropic phi
    std::vector<double> M(d * d, 0.0);
    for (int r = 0; r < d; ++r) M[r * d + r] = a;
    or_phi_matrix_rows(X.data(), G.data(), d, n, M.data(), 0, n, pm.data());
    double err = 0;
    for (long e = 0; e < n * d; ++e) err = std::fmax(err, std::fabs(ph[e] - pm[e]));
    CHECK(err <= 1e-13);
}

int main()
{
    test_plan();
    test_models_vs_oracle();
    test_oracle_paths();
    if (failures) {
        std::fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    std::printf("sanitize_host: all checks passed\n");
    return 0;
}
