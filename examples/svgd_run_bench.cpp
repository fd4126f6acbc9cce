// The headline workload through the reference's C++ API: SVGD::Run on
// BASELINE cfg3 (N = 65536 particles, d = 8, a sum of k = 4 unnormalised
// Gaussians, median-scaled RBF kernel, Adam(0.1, 0.9, 0.999), fp64), with the
// synthetic inputs bench.py uses (splitmix64: X0 = 3 U[-1,1]^d, means
// 3 U[-1,1]^d, cov_c = (1 + 0.25 c) I).  Each timed Run() is `steps` steps
// of SVGD::Step plus its own set/get of the coordinate matrix; the JSON line
// reports the median of `repeats` runs after one warm-up Run (steps of its
// own).  Options (optional): World / Rank / UniqueId are not used here.
//
//   ./svgd_run_bench [n] [d] [k] [steps] [repeats]
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "Core"
#include "Kernel"
#include "Model"
#include "Optimizer"

// bench.py splitmix: element i (1-based counter) -> scale (2u - 1), u in [0, 1)
static std::vector<double> splitmix(size_t count, double scale, uint64_t seed)
{
    std::vector<double> out(count);
    for (size_t i = 0; i < count; ++i)
    {
        uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z = z ^ (z >> 31);
        const double u = (double)(z >> 11) * 0x1.0p-53;
        out[i] = scale * (u * 2.0 - 1.0);
    }
    return out;
}

int main(int argc, char **argv)
{
    const size_t n = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 65536;
    const size_t d = argc > 2 ? std::strtoul(argv[2], nullptr, 10) : 8;
    const size_t k = argc > 3 ? std::strtoul(argv[3], nullptr, 10) : 4;
    const size_t steps = argc > 4 ? std::strtoul(argv[4], nullptr, 10) : 20;
    const size_t repeats = argc > 5 ? std::strtoul(argv[5], nullptr, 10) : 5;

    // particle i at columns i of the d x n col-major matrix == row i of bench.py's (n, d)
    auto particles = std::make_shared<Eigen::MatrixXd>((long)d, (long)n);
    const std::vector<double> x0 = splitmix(n * d, 3.0, 0x5EED), mu = splitmix(k * d, 3.0, 0x5EEE);
    std::copy(x0.begin(), x0.end(), particles->data());
    std::shared_ptr<Model> target;
    for (size_t c = 0; c < k; ++c)
    {
        Eigen::VectorXd m((long)d);
        for (size_t r = 0; r < d; ++r)
            m(r) = mu[c * d + r];
        Eigen::MatrixXd cov = Eigen::MatrixXd::Identity((long)d, (long)d) * (1.0 + 0.25 * (double)c);
        MultivariateNormal comp(m, cov);
        target = target ? std::make_shared<Model>(*target + comp) : std::make_shared<Model>(comp);
    }
    auto kernel = std::make_shared<GaussianRBFKernel>(particles, GaussianRBFKernel::ScaleMethod::Median, target);
    auto optimizer = std::make_shared<Adam>(d, n, 0.1, 0.9, 0.999);

    SVGD svgd(d, steps, particles, kernel, target, optimizer);
    svgd.Initialize();
    svgd.Run(); // warm-up
    std::vector<double> ms;
    for (size_t r = 0; r < repeats; ++r)
    {
        const auto t0 = std::chrono::steady_clock::now();
        svgd.Run();
        ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() /
                     (double)steps);
    }
    std::vector<double> sorted = ms;
    std::sort(sorted.begin(), sorted.end());
    const double med = sorted[sorted.size() / 2];
    double finite = 1.0;
    for (long e = 0; e < particles->size(); ++e)
        finite *= std::isfinite((*particles)(e)) ? 1.0 : 0.0;
    std::printf("{\"metric\": \"particle-updates/s through the C++ SVGD::Run (include/SVGDCpp/SVGD.hpp), "
                "N=%zu d=%zu GMM(k=%zu)\", \"value\": %.6f, \"unit\": \"particle-updates/s\", \"ms_per_step\": %.6f, "
                "\"steps\": %zu, \"repeats\": {\"n\": %zu, \"rule\": \"median Run() of steps steps (its set/get of "
                "the coordinate matrix included)\", \"ms_per_step\": [",
                n, d, k, (double)n / (med / 1e3), med, steps, repeats);
    for (size_t r = 0; r < ms.size(); ++r)
        std::printf("%s%.6f", r ? ", " : "", ms[r]);
    std::printf("]}, \"pipelined_step\": %s, \"dtype\": \"f64\", \"finite\": %s, \"scale_a\": %.17g}\n",
                svgd.UsesPipelinedStep() ? "true" : "false", finite == 1.0 ? "true" : "false", kernel->GetScale());
    return 0;
}
