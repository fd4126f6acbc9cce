// Host gradient timing and agreement of the two block builds
// (host_models.cpp): the 4-particle AVX2 block (variant 1) and the 8-lane
// AVX-512 structure-of-arrays block (variant 2), N particles, d dims, k
// components, T threads; best of 5 runs each.  Linked against host_models.o:
//   g++ -O2 -fopenmp -std=c++17 tools/bench_host_grad.cpp svgdcpp_amd/csrc/host_models.o -o build/host_grad_bench
//   ./build/host_grad_bench [n d k threads]
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../svgdcpp_amd/csrc/host_models.h"
extern "C" int svgd_model_create(void **out, int dim, int ncomp, const double *mus, const double *covs);

int main(int argc, char **argv)
{
    const long n = argc > 1 ? atol(argv[1]) : 65536;
    const int d = argc > 2 ? atoi(argv[2]) : 8, k = argc > 3 ? atoi(argv[3]) : 4;
    const int threads = argc > 4 ? atoi(argv[4]) : 2;
    std::vector<double> X(n * d), mu((size_t)k * d), cov((size_t)k * d * d, 0.0);
    for (int c = 0; c < k; ++c)
        for (int r = 0; r < d; ++r) {
            cov[((size_t)c * d + r) * d + r] = 1.0 + 0.25 * c;
            if (r + 1 < d) cov[((size_t)c * d + r) * d + r + 1] = cov[((size_t)c * d + r + 1) * d + r] = 0.1;
            mu[(size_t)c * d + r] = 0.3 * c - 0.1 * r;
        }
    for (long e = 0; e < n * d; ++e) X[e] = 3.0 * ((double)((e * 2654435761u) % 10007) / 5003.5 - 1.0);
    void *h;
    if (svgd_model_create(&h, d, k, mu.data(), cov.data())) return 1;
    const auto *m = static_cast<const svgd_amd::HostModel *>(h);
    std::vector<double> G[3];
    double best[3] = {0, 0, 0};
    for (int v = 1; v <= 2; ++v) {
        G[v].assign(n * d, 0.0);
        best[v] = 1e30;
        for (int it = 0; it < 5; ++it) {
            auto t = std::chrono::steady_clock::now();
            if (svgd_amd::model_logp_grad_variant(m, X.data(), n, G[v].data(), threads, v)) {
                std::printf("variant %d unavailable on this host\n", v);
                best[v] = -1;
                break;
            }
            best[v] = std::min(best[v], std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count());
        }
    }
    double maxrel = 0.0;
    if (best[2] >= 0)
        for (long e = 0; e < n * d; ++e)
            maxrel = std::max(maxrel, std::fabs(G[1][e] - G[2][e]) / std::max(1e-300, std::fabs(G[1][e]) + 1e-3));
    std::printf("n=%ld d=%d k=%d threads=%d: avx2-block %.3f ms, avx512-soa8 %.3f ms, max rel diff %.3e\n", n, d, k,
                threads, best[1], best[2], maxrel);
    return 0;
}
