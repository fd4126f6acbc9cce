// Host gradient timing (svgd_model_logp_grad): N particles, d dims, k
// components; prints the last of 3 runs.  Usage: host_grad_bench [n d k]
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>
extern "C" int svgd_model_create(void **out, int dim, int ncomp, const double *mus, const double *covs);
extern "C" int svgd_model_logp_grad(void *model, const double *X, int64_t nrows, double *G);
int main(int argc, char **argv)
{
    const long n = argc > 1 ? atol(argv[1]) : 65536;
    const int d = argc > 2 ? atoi(argv[2]) : 64, k = argc > 3 ? atoi(argv[3]) : 1;
    std::vector<double> X(n * d), G(n * d), mu((size_t)k * d), cov((size_t)k * d * d, 0.0);
    for (int c = 0; c < k; ++c)
        for (int r = 0; r < d; ++r) {
            cov[((size_t)c * d + r) * d + r] = 1.0 + 0.25 * c;
            mu[(size_t)c * d + r] = 0.1 * c;
        }
    for (long e = 0; e < n * d; ++e) X[e] = (double)((e * 2654435761u) % 1000) / 500.0 - 1.0;
    void *m;
    svgd_model_create(&m, d, k, mu.data(), cov.data());
    double ms = 0;
    for (int it = 0; it < 3; ++it) {
        auto t = std::chrono::steady_clock::now();
        svgd_model_logp_grad(m, X.data(), n, G.data());
        ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    }
    printf("n=%ld d=%d k=%d: %.3f ms\n", n, d, k, ms);
}
