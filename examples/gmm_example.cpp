// Two-component Gaussian mixture target (MVN + MVN composition) through the
// SVGDCpp-compatible C++ API -- the reference's examples/gaussian_mixture_model
// workload (20 particles, Adam), with the particle count as a knob so the same
// program drives the headline N=65536 configuration on the GPU.
//
//   ./gmm_example [num_particles] [num_iterations]
#include <chrono>
#include <cstdlib>
#include <iostream>

#include "Core"
#include "Kernel"
#include "Model"
#include "Optimizer"

int main(int argc, char **argv)
{
    const size_t dim = 2;
    const size_t n = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 20;
    const size_t iters = argc > 2 ? std::strtoul(argv[2], nullptr, 10) : 1000;

    Eigen::Vector2d mu_a(3.6871, -2.801), mu_b(-2.9802, 4.3387);
    Eigen::Matrix2d cov_a, cov_b;
    cov_a << 0.5001, 0.2426, 0.2426, 0.8420;
    cov_b << 0.6779, -0.1652, -0.1652, 0.2260;
    cov_a *= 5;
    cov_b *= 5;

    MultivariateNormal comp_a(mu_a, cov_a), comp_b(mu_b, cov_b);
    Model mixture = comp_a + comp_b;
    auto target = std::make_shared<Model>(mixture);

    auto particles = std::make_shared<Eigen::MatrixXd>(8 * Eigen::MatrixXd::Random(dim, n));
    if (n <= 64)
        std::cout << "Initial particle coordinates\n" << *particles << "\n";

    auto kernel = std::make_shared<GaussianRBFKernel>(particles, GaussianRBFKernel::ScaleMethod::Median, target);
    auto optimizer = std::make_shared<Adam>(dim, n, 1.0e-1, 0.9, 0.999);

    SVGD svgd(dim, iters, particles, kernel, target, optimizer);
    svgd.Initialize();
    const auto t0 = std::chrono::steady_clock::now();
    svgd.Run();
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();

    if (n <= 64)
        std::cout << "Final particle coordinates\n" << *particles << "\n";
    size_t near_a = 0;
    for (size_t i = 0; i < n; ++i)
    {
        const double da = ((*particles)(0, i) - mu_a(0)) * ((*particles)(0, i) - mu_a(0)) +
                          ((*particles)(1, i) - mu_a(1)) * ((*particles)(1, i) - mu_a(1));
        const double db = ((*particles)(0, i) - mu_b(0)) * ((*particles)(0, i) - mu_b(0)) +
                          ((*particles)(1, i) - mu_b(1)) * ((*particles)(1, i) - mu_b(1));
        near_a += da < db;
    }
    std::cout << "Particles nearer component A: " << near_a << " of " << n << "\n";
    std::cout << "Run: " << iters << " steps x " << n << " particles in " << secs << " s ("
              << (double)iters * (double)n / secs << " particle-updates/s)\n";
    return 0;
}
