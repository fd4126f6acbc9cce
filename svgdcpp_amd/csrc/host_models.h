// Internal layout of the built-in Gaussian-sum model handle (host_models.cpp),
// shared with the C ABI so a context can mirror the model on the device.
#pragma once
#include <vector>

namespace svgd_amd {
struct HostModel {
    int d = 0, k = 0;
    std::vector<double> mu;   // k x d
    std::vector<double> prec; // k x d x d (row-major), inverse covariances
    std::vector<double> precT; // the same, each transposed (prec[c][r][l] at [c][l][r])
};
} // namespace svgd_amd
