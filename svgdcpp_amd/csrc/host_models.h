// Internal layout of the built-in Gaussian-sum model handle (host_models.cpp),
// shared with the C ABI so a context can mirror the model on the device.
#pragma once
#include <cstdint>
#include <vector>

namespace svgd_amd {
struct HostModel {
    int d = 0, k = 0;
    std::vector<double> mu;   // k x d
    std::vector<double> prec; // k x d x d (row-major), inverse covariances
    std::vector<double> precT; // the same, each transposed (prec[c][r][l] at [c][l][r])
};
// svgd_model_logp_grad on nthreads OpenMP threads (<= 0: the OpenMP default)
int model_logp_grad_threads(const HostModel *m, const double *X, int64_t nrows, double *G,
                            int nthreads);
// true when the gradient takes the AVX-512 structure-of-arrays block (~2.5x
// the AVX2 block's rate on the MI355X boxes' EPYC 9575F at d = 8, k = 4)
bool host_grad_avx512();
// A/B and tests: variant 1 the 4-particle block (AVX2 or baseline build),
// 2 the 8-lane structure-of-arrays block (AVX-512 hosts only; else
// SVGD_ERR_ARG), 0 the host's best (what every other call uses)
int model_logp_grad_variant(const HostModel *m, const double *X, int64_t nrows, double *G, int nthreads,
                            int variant);
} // namespace svgd_amd
