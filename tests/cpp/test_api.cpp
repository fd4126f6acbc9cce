// C++ API tests: the SVGDCpp-compatible headers over libsvgdcpp_amd.so.
//
// Follows the reference's tests/test_svgd.cpp strategy (SVGD class vs a
// manual host loop, :9-60 and :66-203) plus the argument checks of
// SVGD.hpp:151-250.  The manual loop is an independent host computation of
// the same step built from the header's host restatements (kernel
// EvaluateKernel/EvaluateKernelGrad, Optimizer::Step, ComputeScale).
//
//   ./test_api cpu   argument/ctor checks that never touch the GPU
//   ./test_api       everything (needs a GPU)
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <string>

#include "Core"
#include "Kernel"
#include "Model"
#include "Optimizer"

static int g_fail = 0, g_pass = 0;
#define CHECK(cond)                                                              \
    do                                                                           \
    {                                                                            \
        if (cond)                                                                \
            ++g_pass;                                                            \
        else                                                                     \
        {                                                                        \
            ++g_fail;                                                            \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
        }                                                                        \
    } while (0)

template <class E, class F>
static bool Throws(F f)
{
    try
    {
        f();
    }
    catch (const E &)
    {
        return true;
    }
    catch (...)
    {
        return false;
    }
    return false;
}

// test_svgd.cpp:78-90 model: p(x) = a cos x0 + b cos x1 + c x0 x1 + d
// (a, b, c, d) = (7.5, 10, 3, -6), written as a host-gradient Model subclass.
class CosineModel : public Model
{
public:
    CosineModel() : Model(2) {}
    double p(const Eigen::VectorXd &x) const
    {
        return a_ * std::cos(x(0)) + b_ * std::cos(x(1)) + c_ * x(0) * x(1) + d_;
    }
    Eigen::VectorXd EvaluateLogModelGrad(const Eigen::VectorXd &x) override
    {
        Eigen::VectorXd g(2);
        g(0) = -a_ * std::sin(x(0)) + c_ * x(1);
        g(1) = -b_ * std::sin(x(1)) + c_ * x(0);
        return g / p(x);
    }

private:
    double a_ = 7.5, b_ = 10.0, c_ = 3.0, d_ = -6.0;
};

// One host step: phi_i = 1/N sum_j [k(x_j, x_i) grad log p(x_j) + grad_{x_j} k(x_j, x_i)],
// x += opt.Step(phi), clamp (test_svgd.cpp:21-60).
static Eigen::MatrixXd ManualStep(const Eigen::MatrixXd &x, Model &model, GaussianRBFKernel &kernel,
                                  Optimizer &opt, const Eigen::VectorXd *lo, const Eigen::VectorXd *hi)
{
    const long d = x.rows(), n = x.cols();
    Eigen::MatrixXd phi = Eigen::MatrixXd::Zero(d, n), grads(d, n);
    for (long j = 0; j < n; ++j)
    {
        Eigen::VectorXd g = model.EvaluateLogModelGrad(x.col(j));
        grads.setCol(j, g);
    }
    for (long i = 0; i < n; ++i)
    {
        kernel.UpdateLocation(x.col(i));
        for (long j = 0; j < n; ++j)
        {
            const Eigen::VectorXd xj = x.col(j);
            const double kv = kernel.EvaluateKernel(xj);
            const Eigen::VectorXd kg = kernel.EvaluateKernelGrad(xj);
            for (long k = 0; k < d; ++k)
                phi(k, i) += kv * grads(k, j) + kg(k);
        }
    }
    phi /= (double)n;
    Eigen::MatrixXd out = x + opt.Step(phi);
    if (lo)
        for (long i = 0; i < n; ++i)
            for (long k = 0; k < d; ++k)
                out(k, i) = std::max(std::min(out(k, i), (*hi)(k)), (*lo)(k));
    return out;
}

static double MaxAbsDiff(const Eigen::MatrixXd &a, const Eigen::MatrixXd &b)
{
    double m = 0.0;
    for (long e = 0; e < a.size(); ++e)
        m = std::max(m, std::fabs(a(e) - b(e)));
    return m;
}

static void TestArgumentChecks()
{
    const size_t d = 2, n = 8;
    auto x = std::make_shared<Eigen::MatrixXd>(Eigen::MatrixXd::Random(d, n));
    std::shared_ptr<Model> model = std::make_shared<MultivariateNormal>(Eigen::Vector2d(0.0, 0.0),
                                                                       Eigen::MatrixXd::Identity(2, 2));
    std::shared_ptr<Kernel> kernel = std::make_shared<GaussianRBFKernel>(x);
    std::shared_ptr<Optimizer> opt = std::make_shared<Adam>(d, n, 0.1, 0.9, 0.999);

    // SVGD.hpp:170-173 dimension check; :223-236 null pointers
    CHECK(Throws<DimensionMismatchException>([&] { SVGD s(3, 1, x, kernel, model, opt); }));
    CHECK(Throws<std::invalid_argument>([&] { SVGD s(d, 1, x, nullptr, model, opt); }));
    CHECK(Throws<std::invalid_argument>([&] { SVGD s(d, 1, x, kernel, nullptr, opt); }));
    CHECK(Throws<std::invalid_argument>([&] { SVGD s(d, 1, x, kernel, model, nullptr); }));
    // bounds of the wrong size (SVGD.hpp:193-207)
    CHECK(Throws<DimensionMismatchException>(
        [&] { SVGD s(d, 1, x, kernel, model, opt, Eigen::VectorXd::Constant(3, -1.0), Eigen::VectorXd::Constant(2, 1.0)); }));
    CHECK(Throws<DimensionMismatchException>(
        [&] { SVGD s(d, 1, x, kernel, model, opt, Eigen::VectorXd::Constant(2, -1.0), Eigen::VectorXd::Constant(5, 1.0)); }));
    // a non-RBF kernel has no device path
    std::shared_ptr<Kernel> plain = std::make_shared<Kernel>(d);
    CHECK(Throws<std::invalid_argument>([&] { SVGD s(d, 1, x, plain, model, opt); }));
    // optimizer parameter checks (Adam.hpp:52-55, RMSProp.hpp:47-50)
    CHECK(Throws<std::invalid_argument>([&] { Adam a(d, n, 0.1, 1.0, 0.999); }));
    CHECK(Throws<std::invalid_argument>([&] { RMSProp r(d, n, 0.1, 1.5); }));
    // model composition checks (Model.hpp:55-92)
    MultivariateNormal m2(Eigen::Vector2d(0.0, 0.0), Eigen::MatrixXd::Identity(2, 2));
    MultivariateNormal m3(Eigen::VectorXd::Zero(3), Eigen::MatrixXd::Identity(3, 3));
    CHECK(Throws<DimensionMismatchException>([&] { Model m = m2 + m3; }));
    CHECK(Throws<DimensionMismatchException>(
        [&] { MultivariateNormal bad(Eigen::VectorXd::Zero(3), Eigen::MatrixXd::Identity(2, 2)); }));
    // host MVN gradient: -Sigma^-1 (x - mu)
    Eigen::Matrix2d cov;
    cov << 2.0, 0.5, 0.5, 1.0;
    MultivariateNormal mvn(Eigen::Vector2d(1.0, -1.0), cov);
    mvn.Initialize();
    const Eigen::VectorXd g = mvn.EvaluateLogModelGrad(Eigen::Vector2d(0.0, 0.0));
    const Eigen::MatrixXd expect = -1.0 * (svgdcpp::Inverse(cov) * (Eigen::Vector2d(0.0, 0.0) - Eigen::Vector2d(1.0, -1.0)));
    CHECK(MaxAbsDiff(g, expect) < 1e-14);
    // Normalisation constant of a 2-D unit Gaussian
    MultivariateNormal unit(Eigen::Vector2d(0.0, 0.0), Eigen::MatrixXd::Identity(2, 2));
    CHECK(std::fabs(unit.GetNormalizationConstant() - 1.0 / (2.0 * M_PI)) < 1e-15);
}

// test_svgd.cpp:66-203: SVGD class (fixed unit scale kernel, custom model,
// Adam, bounds [-1, 1], intermediate-matrix log) vs the manual loop.
static void TestSVGDClassConstantScale()
{
    const size_t d = 2, n = 10, iters = 15;
    std::srand(1);
    auto x = std::make_shared<Eigen::MatrixXd>(Eigen::MatrixXd::Random(d, n));
    const Eigen::MatrixXd x0 = *x;
    auto model = std::make_shared<CosineModel>();
    auto kernel = std::make_shared<GaussianRBFKernel>(x, GaussianRBFKernel::ScaleMethod::Constant);
    kernel->UpdateParameters({Eigen::MatrixXd::Identity(2, 2)});
    auto opt = std::make_shared<Adam>(d, n, 1.0e-1, 0.9, 0.999);
    const Eigen::Vector2d lo(-1.0, -1.0), hi(1.0, 1.0);
    const std::string log_path = "test_api_log.txt";

    SVGDOptions o;
    o.Dimension = d;
    o.NumIterations = iters;
    o.CoordinateMatrixPtr = x;
    o.KernelPtr = kernel;
    o.ModelPtr = model;
    o.OptimizerPtr = opt;
    o.LowerBound = lo;
    o.UpperBound = hi;
    o.LogIntermediateMatrices = true;
    o.IntermediateMatricesOutputPath = log_path;
    SVGD svgd(o);
    CHECK(Throws<UnsetException>([&] { svgd.Run(); }));
    svgd.Initialize();
    svgd.Run();
    CHECK(x->rows() == (long)d && x->cols() == (long)n);

    CosineModel host_model;
    GaussianRBFKernel host_kernel(std::make_shared<Eigen::MatrixXd>(x0), GaussianRBFKernel::ScaleMethod::Constant);
    host_kernel.UpdateParameters({Eigen::MatrixXd::Identity(2, 2)});
    Adam host_opt(d, n, 1.0e-1, 0.9, 0.999);
    host_opt.Initialize();
    Eigen::MatrixXd xm = x0;
    for (size_t t = 0; t < iters; ++t)
        xm = ManualStep(xm, host_model, host_kernel, host_opt, &lo, &hi);
    const double err = MaxAbsDiff(*x, xm);
    std::printf("constant-scale SVGD vs manual loop: max |dx| = %.3e\n", err);
    CHECK(err < 1e-10);
    CHECK(MaxAbsDiff(*x, x0) > 1e-3);
    for (long e = 0; e < x->size(); ++e)
        CHECK((*x)(e) >= -1.0 && (*x)(e) <= 1.0);

    std::ifstream f(log_path);
    std::string text((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    CHECK(text.find("========== Step 1 ==========") != std::string::npos);
    CHECK(text.find("========== Step 15 ==========") != std::string::npos);
    CHECK(text.find("KernelGrad=") != std::string::npos);
    std::remove(log_path.c_str());
}

// Median-heuristic scale + Gaussian mixture + each optimizer vs the manual
// loop with the host median (GaussianRBFKernel.hpp:141-188).
static void TestSVGDMedianGMM(int which)
{
    const size_t d = 2, n = 50, iters = 20;
    std::srand(7 + which);
    auto x = std::make_shared<Eigen::MatrixXd>(6 * Eigen::MatrixXd::Random(d, n));
    const Eigen::MatrixXd x0 = *x;
    Eigen::Matrix2d c1, c2;
    c1 << 0.5001, 0.2426, 0.2426, 0.8420;
    c2 << 0.6779, -0.1652, -0.1652, 0.2260;
    MultivariateNormal a(Eigen::Vector2d(3.6871, -2.801), 5 * c1), b(Eigen::Vector2d(-2.9802, 4.3387), 5 * c2);
    auto model = std::make_shared<Model>(a + b);
    auto kernel = std::make_shared<GaussianRBFKernel>(x, GaussianRBFKernel::ScaleMethod::Median, model);
    std::shared_ptr<Optimizer> opt, host_opt;
    if (which == 0)
    {
        opt = std::make_shared<Adam>(d, n, 1.0e-1, 0.9, 0.999);
        host_opt = std::make_shared<Adam>(d, n, 1.0e-1, 0.9, 0.999);
    }
    else if (which == 1)
    {
        opt = std::make_shared<AdaGrad>(d, n, 1.0e-1);
        host_opt = std::make_shared<AdaGrad>(d, n, 1.0e-1);
    }
    else
    {
        opt = std::make_shared<RMSProp>(d, n, 5.0e-2, 0.9);
        host_opt = std::make_shared<RMSProp>(d, n, 5.0e-2, 0.9);
    }
    SVGD svgd(d, iters, x, kernel, model, opt);
    svgd.Initialize();
    svgd.Run();

    Model host_model = a + b;
    host_model.Initialize();
    auto xm = std::make_shared<Eigen::MatrixXd>(x0);
    GaussianRBFKernel host_kernel(xm, GaussianRBFKernel::ScaleMethod::Median);
    host_opt->Initialize();
    for (size_t t = 0; t < iters; ++t)
    {
        host_kernel.Step(); // host median of the current coordinates
        *xm = ManualStep(*xm, host_model, host_kernel, *host_opt, nullptr, nullptr);
    }
    const double err = MaxAbsDiff(*x, *xm);
    std::printf("median-scale GMM SVGD (optimizer %d) vs manual loop: max |dx| = %.3e\n", which, err);
    CHECK(err < 1e-10);
    // the kernel reports the last device scale
    CHECK(std::fabs(kernel->GetScale() - host_kernel.GetScale()) <= 1e-12 * host_kernel.GetScale());
}

// Hessian scale (GaussianRBFKernel.hpp:189-210) and a constant full-matrix
// scale: SVGD class vs the manual loop with the host kernel's ComputeScale.
static void TestSVGDMatrixScales(bool hessian)
{
    const size_t d = 2, n = 80, iters = 8;
    std::srand(11);
    auto x = std::make_shared<Eigen::MatrixXd>(4 * Eigen::MatrixXd::Random(d, n));
    const Eigen::MatrixXd x0 = *x;
    Eigen::Matrix2d c1, c2;
    c1 << 0.5001, 0.2426, 0.2426, 0.8420;
    c2 << 0.6779, -0.1652, -0.1652, 0.2260;
    MultivariateNormal a(Eigen::Vector2d(1.6871, -0.801), 3 * c1), b(Eigen::Vector2d(-1.9802, 1.3387), 3 * c2);
    auto model = std::make_shared<Model>(a + b);
    Eigen::Matrix2d Mc;
    Mc << 0.30, 0.12, 0.12, 0.55;
    const auto method = hessian ? GaussianRBFKernel::ScaleMethod::Hessian : GaussianRBFKernel::ScaleMethod::Constant;
    auto kernel = std::make_shared<GaussianRBFKernel>(x, method, model);
    if (!hessian)
        kernel->UpdateParameters({Mc});
    auto opt = std::make_shared<Adam>(d, n, 5.0e-2, 0.9, 0.999);
    SVGD svgd(d, iters, x, kernel, model, opt);
    svgd.Initialize();
    svgd.Run();

    Model host_model = a + b;
    host_model.Initialize();
    auto xm = std::make_shared<Eigen::MatrixXd>(x0);
    GaussianRBFKernel host_kernel(xm, method, std::make_shared<Model>(a + b));
    if (!hessian)
        host_kernel.UpdateParameters({Mc});
    Adam host_opt(d, n, 5.0e-2, 0.9, 0.999);
    host_opt.Initialize();
    for (size_t t = 0; t < iters; ++t)
    {
        host_kernel.Step();
        *xm = ManualStep(*xm, host_model, host_kernel, host_opt, nullptr, nullptr);
    }
    const double err = MaxAbsDiff(*x, *xm);
    std::printf("%s-scale SVGD vs manual loop: max |dx| = %.3e\n", hessian ? "Hessian" : "matrix", err);
    CHECK(err < 1e-10);
    CHECK(MaxAbsDiff(kernel->GetScaleMatrix(), host_kernel.GetScaleMatrix()) < 1e-12);
}

int main(int argc, char **argv)
{
    const bool cpu_only = argc > 1 && std::strcmp(argv[1], "cpu") == 0;
    TestArgumentChecks();
    if (!cpu_only)
    {
        TestSVGDClassConstantScale();
        for (int w = 0; w < 3; ++w)
            TestSVGDMedianGMM(w);
        TestSVGDMatrixScales(true);
        TestSVGDMatrixScales(false);
    }
    std::printf("%d checks passed, %d failed\n", g_pass, g_fail);
    return g_fail == 0 ? 0 : 1;
}
