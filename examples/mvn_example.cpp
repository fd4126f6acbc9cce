// Multivariate-normal target through the SVGDCpp-compatible C++ API.
// Mirrors the reference's examples/multivariate_normal (2-D MVN, 10
// particles, AdaGrad, median-scaled RBF kernel); every SVGD step runs on the
// GPU through libsvgdcpp_amd.so.
//
//   ./mvn_example [num_particles] [num_iterations]
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
    const size_t n = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 10;
    const size_t iters = argc > 2 ? std::strtoul(argv[2], nullptr, 10) : 1000;

    Eigen::Vector2d mu(-0.6871, 0.8010);
    Eigen::Matrix2d sigma;
    sigma << 0.2260, 0.1652, 0.1652, 0.6779;
    sigma *= 5;
    std::shared_ptr<Model> target = std::make_shared<MultivariateNormal>(mu, sigma);

    auto particles = std::make_shared<Eigen::MatrixXd>(3 * Eigen::MatrixXd::Random(dim, n));
    if (n <= 64)
        std::cout << "Initial particle coordinates\n" << *particles << "\n";

    auto kernel = std::make_shared<GaussianRBFKernel>(particles, GaussianRBFKernel::ScaleMethod::Median, target);
    auto optimizer = std::make_shared<AdaGrad>(dim, n, 1.0e-1);

    SVGD svgd(dim, iters, particles, kernel, target, optimizer);
    svgd.Initialize();
    const auto t0 = std::chrono::steady_clock::now();
    svgd.Run();
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();

    if (n <= 64)
        std::cout << "Final particle coordinates\n" << *particles << "\n";
    Eigen::VectorXd mean = Eigen::VectorXd::Zero(dim);
    for (size_t i = 0; i < n; ++i)
        for (size_t k = 0; k < dim; ++k)
            mean(k) += (*particles)(k, i) / (double)n;
    std::cout << "Particle mean " << mean.transpose() << " (target " << mu.transpose() << ")\n";
    std::cout << "Kernel scale after the last step " << kernel->GetScale() << "\n";
    std::cout << "Run: " << iters << " steps x " << n << " particles in " << secs << " s\n";
    return 0;
}
