// A sharded SVGD::Run through the C++ API (SVGDOptions World / Rank): one
// process per rank, collectives through the host shared-memory rehearsal
// backend (SVGD_HOSTCOMM, set by tests/test_cpp_api.py; all ranks on one
// GPU).  Every rank passes the full coordinate matrix and ends with all of
// it; rank r writes it (n x d doubles, particle-contiguous) to out.
//
//   ./test_dist world rank n d steps out [pipelined 1|0]
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "Core"
#include "Kernel"
#include "Model"
#include "Optimizer"

// a user model that is not a built-in Gaussian form: the split begin /
// gradient / finish calls on this rank's rows
class ShiftedMvn : public MultivariateNormal
{
public:
    using MultivariateNormal::MultivariateNormal;
    std::shared_ptr<Model> CloneSharedPointer() const override { return std::make_shared<ShiftedMvn>(*this); }
};

int main(int argc, char **argv)
{
    if (argc < 7)
        return 2;
    const int world = std::atoi(argv[1]), rank = std::atoi(argv[2]);
    const size_t n = std::strtoul(argv[3], nullptr, 10), d = std::strtoul(argv[4], nullptr, 10);
    const size_t steps = std::strtoul(argv[5], nullptr, 10);
    const bool pipelined = argc < 8 || std::atoi(argv[7]) != 0;

    std::srand(7);
    auto particles = std::make_shared<Eigen::MatrixXd>(3 * Eigen::MatrixXd::Random((long)d, (long)n));
    Eigen::VectorXd mu0((long)d), mu1((long)d);
    for (size_t r = 0; r < d; ++r)
    {
        mu0(r) = 1.0 - 0.3 * (double)r;
        mu1(r) = -0.5 + 0.2 * (double)r;
    }
    const Eigen::MatrixXd cov0 = Eigen::MatrixXd::Identity((long)d, (long)d);
    const Eigen::MatrixXd cov1 = Eigen::MatrixXd::Identity((long)d, (long)d) * 1.5;
    std::shared_ptr<Model> target;
    if (pipelined)
        target = std::make_shared<Model>(MultivariateNormal(mu0, cov0) + MultivariateNormal(mu1, cov1));
    else
        target = std::make_shared<ShiftedMvn>(mu0, cov0);

    SVGDOptions o;
    o.Dimension = d;
    o.NumIterations = steps;
    o.CoordinateMatrixPtr = particles;
    o.ModelPtr = target;
    o.KernelPtr = std::make_shared<GaussianRBFKernel>(particles, GaussianRBFKernel::ScaleMethod::Median, target);
    o.OptimizerPtr = std::make_shared<Adam>(d, n, 0.05, 0.9, 0.999);
    o.LowerBound = Eigen::VectorXd::Constant((long)d, -2.5);
    o.UpperBound = Eigen::VectorXd::Constant((long)d, 2.5);
    o.World = world;
    o.Rank = rank;
    SVGD svgd(o);
    if (svgd.UsesPipelinedStep() != pipelined)
    {
        std::fprintf(stderr, "unexpected step path\n");
        return 3;
    }
    svgd.Initialize();
    svgd.Run();
    std::FILE *f = std::fopen(argv[6], "wb");
    if (!f)
        return 4;
    std::fwrite(particles->data(), sizeof(double), n * d, f);
    std::fclose(f);
    std::printf("rank %d rows [%lld, %lld)\n", rank, (long long)svgd.ShardBegin(), (long long)svgd.ShardEnd());
    return 0;
}
