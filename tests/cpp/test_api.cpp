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
static Eigen::MatrixXd ManualStep(const Eigen::MatrixXd &x, Model &model, Kernel &kernel,
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
    // a kernel with neither a function nor overrides is unset (Kernel.hpp:393-396)
    std::shared_ptr<Kernel> plain = std::make_shared<Kernel>(d);
    CHECK(Throws<UnsetException>([&] { plain->EvaluateKernel(Eigen::Vector2d(0.0, 0.0)); }));
    {
        SVGD s(d, 1, x, plain, model, opt);
        CHECK(!s.UsesDevicePath());
        s.Initialize();
        CHECK(Throws<UnsetException>([&] { s.Run(); }));
    }
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

// exp(-|x - x'|^2) as a closed-form generic kernel (test_svgd.cpp:92-103 +
// its gradient :155-162), and an inverse multiquadric (c^2 + |x - x'|^2)^beta
// derived class overriding EvaluateKernel/EvaluateKernelGrad (Kernel.hpp:279-297).
static std::shared_ptr<Kernel> UnitRBF(size_t d)
{
    auto k = std::make_shared<Kernel>(d);
    k->UpdateKernel(
        [](const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &, const Eigen::VectorXd &loc) {
            const Eigen::VectorXd diff = x - loc;
            return std::exp(-diff.squaredNorm());
        },
        [](const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &, const Eigen::VectorXd &loc) {
            const Eigen::VectorXd diff = x - loc;
            return Eigen::VectorXd(diff * (-2.0 * std::exp(-diff.squaredNorm())));
        });
    return k;
}

class IMQKernel : public Kernel
{
public:
    IMQKernel(size_t d, double c, double beta) : Kernel(d), c_(c), beta_(beta) {}
    std::unique_ptr<Kernel> CloneUniquePointer() const override { return std::make_unique<IMQKernel>(*this); }
    double EvaluateKernel(const Eigen::VectorXd &x) override
    {
        return std::pow(c_ * c_ + (x - location_).squaredNorm(), beta_);
    }
    Eigen::VectorXd EvaluateKernelGrad(const Eigen::VectorXd &x) override
    {
        const Eigen::VectorXd diff = x - location_;
        const double s = c_ * c_ + diff.squaredNorm();
        return Eigen::VectorXd(diff * (2.0 * beta_ * std::pow(s, beta_ - 1.0)));
    }

private:
    double c_, beta_;
};

// Generic kernels on the host path: the SVGD class vs the
// manual loop of test_svgd.cpp:21-60 (15 Adam steps, bounds [-1, 1], the
// reference's own fixed-kernel scenario :66-203), with a closed-form kernel,
// a derived override and a composed kernel; no GPU involved.
static void TestGenericKernelHostPath()
{
    const size_t d = 2, n = 10, iters = 15;
    const Eigen::Vector2d lo(-1.0, -1.0), hi(1.0, 1.0);
    for (int variant = 0; variant < 3; ++variant)
    {
        std::srand(1);
        auto x = std::make_shared<Eigen::MatrixXd>(Eigen::MatrixXd::Random(d, n));
        const Eigen::MatrixXd x0 = *x;
        std::shared_ptr<Kernel> kernel, host;
        if (variant == 0)
        {
            kernel = UnitRBF(d);
            host = UnitRBF(d);
        }
        else if (variant == 1)
        {
            kernel = std::make_shared<IMQKernel>(d, 1.0, -0.5);
            host = std::make_shared<IMQKernel>(d, 1.0, -0.5);
        }
        else
        {
            kernel = std::make_shared<Kernel>(*UnitRBF(d) * *UnitRBF(d) + *UnitRBF(d));
            host = std::make_shared<Kernel>(*UnitRBF(d) * *UnitRBF(d) + *UnitRBF(d));
        }
        auto model = std::make_shared<CosineModel>();
        auto opt = std::make_shared<Adam>(d, n, 1.0e-1, 0.9, 0.999);
        SVGDOptions o;
        o.Dimension = d;
        o.NumIterations = iters;
        o.CoordinateMatrixPtr = x;
        o.KernelPtr = kernel;
        o.ModelPtr = model;
        o.OptimizerPtr = opt;
        o.LowerBound = lo;
        o.UpperBound = hi;
        SVGD svgd(o);
        CHECK(!svgd.UsesDevicePath() && svgd.Context() == nullptr);
        svgd.Initialize();
        svgd.Run();
        CosineModel host_model;
        Adam host_opt(d, n, 1.0e-1, 0.9, 0.999);
        host_opt.Initialize();
        Eigen::MatrixXd xm = x0;
        for (size_t t = 0; t < iters; ++t)
            xm = ManualStep(xm, host_model, *host, host_opt, &lo, &hi);
        const double err = MaxAbsDiff(*x, xm);
        std::printf("generic kernel %d (host path) vs manual loop: max |dx| = %.3e\n", variant, err);
        CHECK(err < 1e-12);
        CHECK(MaxAbsDiff(*x, x0) > 1e-3);
    }
    // composition rules vs the operands (Kernel.hpp:55-223) and a central
    // finite difference of the composed gradient
    Kernel a = *UnitRBF(2), b = *UnitRBF(2);
    b.UpdateKernel(
        [](const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &p, const Eigen::VectorXd &loc) {
            return 1.0 + p.at(0)(0, 0) * (x - loc).squaredNorm();
        },
        [](const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &p, const Eigen::VectorXd &loc) {
            return Eigen::VectorXd((x - loc) * (2.0 * p.at(0)(0, 0)));
        });
    b.UpdateParameters({Eigen::MatrixXd::Constant(1, 1, 0.7)});
    const Eigen::Vector2d loc(0.2, -0.4), x1(0.5, 0.3);
    Kernel ops[4] = {a + b, a - b, a * b, a / b};
    a.UpdateLocation(loc);
    b.UpdateLocation(loc);
    const double ka = a.EvaluateKernel(x1), kb = b.EvaluateKernel(x1);
    const double expect[4] = {ka + kb, ka - kb, ka * kb, ka / kb};
    for (int q = 0; q < 4; ++q)
    {
        Kernel &k = ops[q];
        CHECK(k.GetParameters().size() == 1);
        k.UpdateLocation(loc);
        CHECK(std::fabs(k.EvaluateKernel(x1) - expect[q]) < 1e-15);
        const Eigen::VectorXd g = k.EvaluateKernelGrad(x1);
        for (long c = 0; c < 2; ++c)
        {
            Eigen::VectorXd xp = x1, xm = x1;
            xp(c) += 1e-6;
            xm(c) -= 1e-6;
            CHECK(std::fabs(g(c) - (k.EvaluateKernel(xp) - k.EvaluateKernel(xm)) / 2e-6) < 1e-8);
        }
    }
    Kernel k3(3);
    CHECK(Throws<DimensionMismatchException>([&] { Kernel s = a + k3; }));
    Kernel unset(2);
    CHECK(Throws<UnsetException>([&] { Kernel s = a + unset; }));

    // a GaussianRBFKernel composes like any set kernel (its constructor sets
    // the closed form, as the reference's sets its lambda,
    // GaussianRBFKernel.hpp:75-87): rbf (+ - * /) b against the operands
    {
        auto xr = std::make_shared<Eigen::MatrixXd>(Eigen::MatrixXd::Random(2, 4));
        GaussianRBFKernel rbf(xr, GaussianRBFKernel::ScaleMethod::Constant);
        Eigen::Matrix2d M;
        M << 0.5, 0.1, 0.1, 0.8;
        rbf.UpdateParameters({Eigen::MatrixXd(M)});
        Kernel rops[4] = {rbf + b, rbf - b, rbf * b, rbf / b};
        rbf.UpdateLocation(loc);
        const Eigen::VectorXd d1 = x1 - loc;
        const double kr = std::exp(-(d1(0) * (M(0, 0) * d1(0) + M(0, 1) * d1(1)) +
                                     d1(1) * (M(1, 0) * d1(0) + M(1, 1) * d1(1))));
        CHECK(std::fabs(rbf.EvaluateKernel(x1) - kr) < 1e-15);
        const double rexp[4] = {kr + kb, kr - kb, kr * kb, kr / kb};
        for (int q = 0; q < 4; ++q)
        {
            Kernel &k = rops[q];
            CHECK(k.GetParameters().size() == 2);
            k.UpdateLocation(loc);
            CHECK(std::fabs(k.EvaluateKernel(x1) - rexp[q]) < 1e-15);
            const Eigen::VectorXd g = k.EvaluateKernelGrad(x1);
            for (long c = 0; c < 2; ++c)
            {
                Eigen::VectorXd xp = x1, xm = x1;
                xp(c) += 1e-6;
                xm(c) -= 1e-6;
                CHECK(std::fabs(g(c) - (k.EvaluateKernel(xp) - k.EvaluateKernel(xm)) / 2e-6) < 1e-8);
            }
        }
    }

    // Parallel = true: the composed kernel on OpenMP threads matches the
    // serial run, and an unset kernel surfaces UnsetException from Run()
    // instead of terminating inside the parallel region
    {
        std::srand(3);
        auto xs = std::make_shared<Eigen::MatrixXd>(Eigen::MatrixXd::Random(2, 12));
        auto xp = std::make_shared<Eigen::MatrixXd>(*xs);
        auto model = std::make_shared<CosineModel>();
        auto mk = [&](const std::shared_ptr<Eigen::MatrixXd> &x, bool par) {
            auto k = std::make_shared<Kernel>(*UnitRBF(2) * *UnitRBF(2) + *UnitRBF(2));
            auto opt = std::make_shared<Adam>(2, 12, 1.0e-1, 0.9, 0.999);
            SVGD s(2, 5, x, k, model, opt, par);
            s.Initialize();
            s.Run();
        };
        mk(xs, false);
        mk(xp, true);
        CHECK(MaxAbsDiff(*xs, *xp) == 0.0);
        std::shared_ptr<Kernel> plain = std::make_shared<Kernel>(2);
        auto opt = std::make_shared<Adam>(2, 12, 1.0e-1, 0.9, 0.999);
        SVGD s(2, 1, xs, plain, model, opt, true);
        s.Initialize();
        CHECK(Throws<UnsetException>([&] { s.Run(); }));
        // the sharding options belong to the device path: a generic kernel
        // with World > 1 or a unique id is refused, not silently unsharded
        SVGDOptions o;
        o.Dimension = 2;
        o.NumIterations = 1;
        o.CoordinateMatrixPtr = xs;
        o.KernelPtr = std::make_shared<Kernel>(*UnitRBF(2) + *UnitRBF(2));
        o.ModelPtr = model;
        o.OptimizerPtr = opt;
        o.World = 2;
        o.Rank = 1;
        CHECK(Throws<std::invalid_argument>([&] { SVGD bad(o); }));
        o.World = 1;
        o.Rank = 0;
        o.UniqueId.assign(128, 0);
        CHECK(Throws<std::invalid_argument>([&] { SVGD bad(o); }));
    }
}

// Model composition over closed forms (reference tests/test_model.cpp:186-315:
// the same functions, compositions and hand-derived values; gradients and
// Hessians also against central differences).
static const Eigen::VectorXd &LowX()
{
    static Eigen::VectorXd x = Eigen::Vector2d(0.7, -1.3);
    return x;
}

static std::vector<Eigen::MatrixXd> CompParams()
{
    Eigen::Matrix2d P;
    P << 2.0, 0.3, -0.1, 1.5; // not symmetric: grad x^T P x = (P + P^T) x
    return {Eigen::MatrixXd(Eigen::Vector2d(1.5, -0.4)), Eigen::MatrixXd(P)};
}

static Model LinearModel() // test_model.cpp:60-67: sum(p .* x)
{
    Model m(2);
    m.UpdateModel([](const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &p)
                  { return p[0](0) * x(0) + p[0](1) * x(1); },
                  [](const Eigen::VectorXd &, const std::vector<Eigen::MatrixXd> &p)
                  { return Eigen::VectorXd(p[0]); },
                  [](const Eigen::VectorXd &, const std::vector<Eigen::MatrixXd> &)
                  { return Eigen::MatrixXd(Eigen::MatrixXd::Zero(2, 2)); });
    m.UpdateParameters(CompParams());
    return m;
}

static Model SquaredModel() // test_model.cpp:69-76: x^T P x
{
    Model m(2);
    m.UpdateModel([](const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &p)
                  { return (x.transpose() * p[1] * x)(0, 0); },
                  [](const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &p)
                  { return Eigen::VectorXd((p[1] + p[1].transpose()) * x); },
                  [](const Eigen::VectorXd &, const std::vector<Eigen::MatrixXd> &p)
                  { return Eigen::MatrixXd(p[1] + p[1].transpose()); });
    m.UpdateParameters(CompParams());
    return m;
}

static Model SumModel(double scale) // test_model.cpp:78-85 (scale 1) and :203-209 (scale 2): scale * sum(x)
{
    Model m(5);
    m.UpdateModel([scale](const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &)
                  {
                      double s = 0.0;
                      for (long k = 0; k < x.rows(); ++k)
                          s += x(k);
                      return scale * s;
                  },
                  [scale](const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &)
                  { return Eigen::VectorXd(Eigen::VectorXd::Constant(x.rows(), scale)); },
                  [](const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &)
                  { return Eigen::MatrixXd(Eigen::MatrixXd::Zero(x.rows(), x.rows())); });
    return m;
}

// "Method 3" (doc/instructions.md:234-301): a derived model with its own
// closed forms, p(x) = 1 + (x0 - 0.5)^2 + x0 x1^2, that composes through
// CloneSharedPointer.
class ShiftedQuad : public Model
{
public:
    ShiftedQuad() : Model(2) {}
    std::shared_ptr<Model> CloneSharedPointer() const override { return std::make_shared<ShiftedQuad>(*this); }
    double EvaluateModel(const Eigen::VectorXd &x) override
    {
        return 1.0 + (x(0) - 0.5) * (x(0) - 0.5) + x(0) * x(1) * x(1);
    }
    Eigen::VectorXd EvaluateModelGrad(const Eigen::VectorXd &x) override
    {
        return Eigen::Vector2d(2.0 * (x(0) - 0.5) + x(1) * x(1), 2.0 * x(0) * x(1));
    }
    Eigen::MatrixXd EvaluateModelHessian(const Eigen::VectorXd &x) override
    {
        Eigen::Matrix2d H;
        H << 2.0, 2.0 * x(1), 2.0 * x(1), 2.0 * x(0);
        return H;
    }
};

// the same closed forms without a CloneSharedPointer override: composing it
// would slice it to a base Model, so the composition refuses it at once
class NoCloneQuad : public Model
{
public:
    NoCloneQuad() : Model(2) {}
    double EvaluateModel(const Eigen::VectorXd &x) override { return 1.0 + x(0) * x(0); }
    Eigen::VectorXd EvaluateModelGrad(const Eigen::VectorXd &x) override { return Eigen::Vector2d(2.0 * x(0), 0.0); }
};

// a derived model that only sets its functions with UpdateModel in its
// constructor (no overrides): slicing it to a base Model keeps them, so it
// composes without a CloneSharedPointer override
class SetFunQuad : public Model
{
public:
    SetFunQuad() : Model(2)
    {
        using P = std::vector<Eigen::MatrixXd>;
        UpdateModel([](const Eigen::VectorXd &x, const P &) { return 2.0 + x(1) * x(1); },
                    [](const Eigen::VectorXd &x, const P &) { return Eigen::VectorXd(Eigen::Vector2d(0.0, 2.0 * x(1))); },
                    [](const Eigen::VectorXd &, const P &)
                    {
                        Eigen::MatrixXd H = Eigen::MatrixXd::Zero(2, 2);
                        H(1, 1) = 2.0;
                        return H;
                    });
    }
};

// grad (and Hessian) of m at x against central differences of the level below
static void CheckDerivatives(Model &m, const Eigen::VectorXd &x, bool hess)
{
    const double h = 1e-5;
    const Eigen::VectorXd g = m.EvaluateModelGrad(x), lg = m.EvaluateLogModelGrad(x);
    const Eigen::MatrixXd H = m.EvaluateModelHessian(x), LH = m.EvaluateLogModelHessian(x);
    for (long c = 0; c < x.rows(); ++c)
    {
        Eigen::VectorXd xp = x, xm = x;
        xp(c) += h;
        xm(c) -= h;
        const double fd = (m.EvaluateModel(xp) - m.EvaluateModel(xm)) / (2 * h);
        CHECK(std::fabs(g(c) - fd) <= 1e-7 * std::max(1.0, std::fabs(fd)));
        const double lfd = (m.EvaluateLogModel(xp) - m.EvaluateLogModel(xm)) / (2 * h);
        CHECK(std::fabs(lg(c) - lfd) <= 1e-7 * std::max(1.0, std::fabs(lfd)));
        if (!hess)
            continue;
        const Eigen::VectorXd gp = m.EvaluateModelGrad(xp), gm = m.EvaluateModelGrad(xm);
        const Eigen::VectorXd lgp = m.EvaluateLogModelGrad(xp), lgm = m.EvaluateLogModelGrad(xm);
        for (long r = 0; r < x.rows(); ++r)
        {
            const double hfd = (gp(r) - gm(r)) / (2 * h), lhfd = (lgp(r) - lgm(r)) / (2 * h);
            CHECK(std::fabs(H(r, c) - hfd) <= 1e-6 * std::max(1.0, std::fabs(hfd)));
            CHECK(std::fabs(LH(r, c) - lhfd) <= 1e-6 * std::max(1.0, std::fabs(lhfd)));
        }
    }
}

static void TestModelComposition()
{
    const Eigen::VectorXd xl = LowX();
    Eigen::VectorXd xh(5);
    xh << 0.3, -0.2, 1.1, 0.4, 0.25;
    const std::vector<Eigen::MatrixXd> p = CompParams();
    const Eigen::VectorXd pv = Eigen::VectorXd(p[0]);
    const Eigen::MatrixXd P = p[1], Ps = P + P.transpose();
    Model lin = LinearModel(), sq = SquaredModel(), hi = SumModel(1.0), hi2 = SumModel(2.0);

    // test_model.cpp:190-193: dimension mismatch
    CHECK(Throws<DimensionMismatchException>([&] { Model s = lin + hi; }));
    CHECK(Throws<DimensionMismatchException>([&] { Model s = lin * hi; }));
    CHECK(Throws<DimensionMismatchException>([&] { Model s = lin - hi; }));
    CHECK(Throws<DimensionMismatchException>([&] { Model s = lin / hi; }));
    Model unset(2);
    CHECK(Throws<UnsetException>([&] { Model s = lin + unset; }));
    CHECK(Throws<UnsetException>([&] { unset.EvaluateModel(xl); }));

    // test_model.cpp:206-233: the compositions and their values
    Model sum1 = lin + lin, sum2 = lin + sq, diff = sq - lin, prod = hi * hi, quot = hi / hi2;
    for (Model *m : {&sum1, &sum2, &diff, &prod, &quot})
        m->Initialize();
    const double lv = pv(0) * xl(0) + pv(1) * xl(1), qv = (xl.transpose() * P * xl)(0, 0);
    double sx = 0.0;
    for (long k = 0; k < 5; ++k)
        sx += xh(k);
    CHECK(std::fabs(sum1.EvaluateModel(xl) - 2 * lv) < 1e-14);
    CHECK(std::fabs(sum2.EvaluateModel(xl) - (lv + qv)) < 1e-14);
    CHECK(std::fabs(diff.EvaluateModel(xl) - (qv - lv)) < 1e-14);
    CHECK(std::fabs(prod.EvaluateModel(xh) - sx * sx) < 1e-14);
    CHECK(std::fabs(quot.EvaluateModel(xh) - 0.5) < 1e-15);

    // hand-derived gradients and Hessians (test_model.cpp:246-315's closed forms, composed)
    CHECK(MaxAbsDiff(sum1.EvaluateModelGrad(xl), 2.0 * pv) < 1e-14);
    CHECK(MaxAbsDiff(sum2.EvaluateModelGrad(xl), Eigen::VectorXd(pv + Ps * xl)) < 1e-14);
    CHECK(MaxAbsDiff(diff.EvaluateModelGrad(xl), Eigen::VectorXd(Ps * xl - pv)) < 1e-14);
    CHECK(MaxAbsDiff(prod.EvaluateModelGrad(xh), Eigen::VectorXd(Eigen::VectorXd::Constant(5, 2.0 * sx))) < 1e-14);
    CHECK(MaxAbsDiff(quot.EvaluateModelGrad(xh), Eigen::VectorXd(Eigen::VectorXd::Zero(5))) < 1e-15);
    CHECK(MaxAbsDiff(sum2.EvaluateModelHessian(xl), Ps) < 1e-14);
    CHECK(MaxAbsDiff(prod.EvaluateModelHessian(xh), Eigen::MatrixXd(Eigen::MatrixXd::Constant(5, 5, 2.0))) < 1e-14);
    CHECK(MaxAbsDiff(quot.EvaluateModelHessian(xh), Eigen::MatrixXd(Eigen::MatrixXd::Zero(5, 5))) < 1e-15);
    // grad log p = grad p / p, hess log p = hess p / p - grad p grad p^T / p^2
    const Eigen::VectorXd g2 = pv + Ps * xl;
    CHECK(MaxAbsDiff(sum2.EvaluateLogModelGrad(xl), Eigen::VectorXd(g2 / (lv + qv))) < 1e-14);
    CHECK(MaxAbsDiff(sum2.EvaluateLogModelHessian(xl),
                     Eigen::MatrixXd(Ps / (lv + qv) - (g2 * g2.transpose()) / ((lv + qv) * (lv + qv)))) < 1e-13);
    CHECK(std::fabs(sum2.EvaluateLogModel(xl) - std::log(lv + qv)) < 1e-14);

    // parameters concatenate (test_model.cpp:70-74) and update the operands
    CHECK(sum2.GetParameters().size() == 4);
    std::vector<Eigen::MatrixXd> q = sum2.GetParameters();
    q[0] = Eigen::MatrixXd(Eigen::Vector2d(3.0, 1.0));
    sum2.UpdateParameters(q);
    CHECK(std::fabs(sum2.EvaluateModel(xl) - (3.0 * xl(0) + xl(1) + qv)) < 1e-14);
    CHECK(std::fabs(lin.EvaluateModel(xl) - lv) < 1e-15); // the operand itself is untouched
    CHECK(Throws<DimensionMismatchException>([&] { sum2.UpdateParameters({p[0]}); }));

    // method-3 derived models compose (through CloneSharedPointer), also
    // with Gaussian forms and inside deeper compositions
    ShiftedQuad sqd;
    NoCloneQuad ncq;
    CHECK(Throws<std::invalid_argument>([&] { Model bad = ncq + lin; }));
    CHECK(Throws<std::invalid_argument>([&] { Model bad = lin * ncq; }));
    {
        SetFunQuad sfq;
        Model ok1 = sfq + lin, ok2 = lin * sfq;
        ok1.Initialize();
        ok2.Initialize();
        const double fv = 2.0 + xl(1) * xl(1);
        CHECK(std::fabs(ok1.EvaluateModel(xl) - (fv + lv)) < 1e-14);
        CHECK(std::fabs(ok2.EvaluateModel(xl) - lv * fv) < 1e-14);
        CheckDerivatives(ok1, xl, true);
    }
    Eigen::Matrix2d cov;
    cov << 1.2, 0.3, 0.3, 0.8;
    MultivariateNormal mvn(Eigen::Vector2d(0.2, -0.1), cov);
    Model mix1 = sqd * mvn, mix2 = (sqd + lin) / sqd, mix3 = sqd * sq - mvn, mix4 = sqd + mvn;
    CHECK(!mix1.IsGaussianForm() && !mix4.IsGaussianForm() && mvn.IsGaussianForm());
    for (Model *m : {&mix1, &mix2, &mix3, &mix4, &sum1, &sum2, &diff})
        CheckDerivatives(*m, xl, true);
    CheckDerivatives(prod, xh, true);
    CheckDerivatives(quot, xh, true);
    CHECK(std::fabs(mix1.EvaluateModel(xl) - sqd.EvaluateModel(xl) * mvn.EvaluateModel(xl)) < 1e-15);

    // the Gaussian fast path is unchanged: MVN + MVN stays a Gaussian form
    // (the batched host kernel) and equals the same sum composed in closed
    // form from function models of the two densities
    Eigen::Matrix2d cov2;
    cov2 << 0.5, -0.1, -0.1, 0.9;
    MultivariateNormal mvn2(Eigen::Vector2d(-0.6, 0.4), cov2);
    Model gsum = mvn + mvn2;
    CHECK(gsum.IsGaussianForm());
    auto wrap = [](const MultivariateNormal &g) {
        auto gp = std::make_shared<MultivariateNormal>(g);
        Model w(2);
        w.UpdateModel([gp](const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &)
                      { return gp->EvaluateModel(x); },
                      [gp](const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &)
                      { return gp->EvaluateModelGrad(x); },
                      [gp](const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &)
                      { return gp->EvaluateModelHessian(x); });
        return w;
    };
    Model fsum = wrap(mvn) + wrap(mvn2);
    CHECK(!fsum.IsGaussianForm());
    for (const Eigen::VectorXd &x : {LowX(), Eigen::VectorXd(Eigen::Vector2d(-0.4, 0.9))})
    {
        CHECK(MaxAbsDiff(gsum.EvaluateLogModelGrad(x), fsum.EvaluateLogModelGrad(x)) < 1e-12);
        CHECK(MaxAbsDiff(gsum.EvaluateLogModelHessian(x), fsum.EvaluateLogModelHessian(x)) < 1e-11);
        CHECK(std::fabs(gsum.EvaluateModel(x) - fsum.EvaluateModel(x)) < 1e-15);
    }
}

// A composed (closed-form) model on the host-gradient path of the device
// step: the same density as a Gaussian form (the batched fast path) gives
// the same trajectory.
static void TestComposedModelSVGD()
{
    const size_t d = 2, n = 300;
    Eigen::Matrix2d c1, c2;
    c1 << 0.5, 0.1, 0.1, 0.7;
    c2 << 0.9, -0.2, -0.2, 0.4;
    auto g1 = std::make_shared<MultivariateNormal>(Eigen::Vector2d(-1.0, 0.5), c1);
    auto g2 = std::make_shared<MultivariateNormal>(Eigen::Vector2d(0.8, -0.3), c2);
    auto fast = std::make_shared<Model>(*g1 + *g2);
    auto wrap = [](const std::shared_ptr<MultivariateNormal> &g) {
        Model w(2);
        w.UpdateModel([g](const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &) { return g->EvaluateModel(x); },
                      [g](const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &) { return g->EvaluateModelGrad(x); });
        return w;
    };
    auto composed = std::make_shared<Model>(wrap(g1) + wrap(g2));
    std::srand(5);
    const Eigen::MatrixXd x0 = 2.0 * Eigen::MatrixXd::Random(d, n);
    Eigen::MatrixXd out[2];
    for (int w = 0; w < 2; ++w)
    {
        auto x = std::make_shared<Eigen::MatrixXd>(x0);
        std::shared_ptr<Model> model = w ? std::static_pointer_cast<Model>(composed) : fast;
        auto kernel = std::make_shared<GaussianRBFKernel>(x, GaussianRBFKernel::ScaleMethod::Median, model);
        auto opt = std::make_shared<Adam>(d, n, 5.0e-2, 0.9, 0.999);
        SVGD svgd(d, 10, x, kernel, model, opt);
        svgd.Initialize();
        svgd.Run();
        out[w] = *x;
    }
    CHECK(MaxAbsDiff(out[0], out[1]) < 1e-10);
    CHECK(MaxAbsDiff(out[0], x0) > 1e-3);
}

// Logged-matrix runs for tests/test_cpp_api.py (value parity of the
// intermediate-matrix log, SVGD.hpp:345-365, against the oracle):
//   host   generic closed-form unit RBF (host path), test_svgd.cpp scenario
//   const  GaussianRBFKernel, Constant M = I (device path), same scenario
//   median GaussianRBFKernel, Median scale (device path), MVN model
// Each writes its log at 17 significant digits and prints the initial and
// final coordinates.
static int LogRun(const std::string &which, const std::string &path)
{
    const size_t d = 2, n = 10, iters = which == "median" ? 5 : 15;
    std::srand(1);
    auto x = std::make_shared<Eigen::MatrixXd>(Eigen::MatrixXd::Random(d, n));
    const Eigen::MatrixXd x0 = *x;
    std::shared_ptr<Model> model = std::make_shared<CosineModel>();
    std::shared_ptr<Kernel> kernel;
    if (which == "host")
        kernel = UnitRBF(d);
    else if (which == "const")
    {
        auto k = std::make_shared<GaussianRBFKernel>(x, GaussianRBFKernel::ScaleMethod::Constant);
        k->UpdateParameters({Eigen::MatrixXd::Identity(2, 2)});
        kernel = k;
    }
    else
    {
        Eigen::Matrix2d cov;
        cov << 0.2260, 0.1652, 0.1652, 0.6779;
        model = std::make_shared<MultivariateNormal>(Eigen::Vector2d(-0.6871, 0.8010), 5.0 * cov);
        kernel = std::make_shared<GaussianRBFKernel>(x, GaussianRBFKernel::ScaleMethod::Median, model);
    }
    SVGDOptions o;
    o.Dimension = d;
    o.NumIterations = iters;
    o.CoordinateMatrixPtr = x;
    o.KernelPtr = kernel;
    o.ModelPtr = model;
    o.OptimizerPtr = std::make_shared<Adam>(d, n, 1.0e-1, 0.9, 0.999);
    if (which != "median")
    {
        o.LowerBound = Eigen::Vector2d(-1.0, -1.0);
        o.UpperBound = Eigen::Vector2d(1.0, 1.0);
    }
    o.LogIntermediateMatrices = true;
    o.IntermediateMatricesOutputPath = path;
    o.IntermediateMatricesPrecision = 17;
    SVGD svgd(o);
    svgd.Initialize();
    svgd.Run();
    std::cout.precision(17);
    std::cout << "INITIAL\n" << x0 << "\nFINAL\n" << *x << "\n";
    return 0;
}

int main(int argc, char **argv)
{
    if (argc > 3 && std::strcmp(argv[1], "log") == 0)
        return LogRun(argv[2], argv[3]);
    const bool cpu_only = argc > 1 && std::strcmp(argv[1], "cpu") == 0;
    TestArgumentChecks();
    TestGenericKernelHostPath();
    TestModelComposition();
    if (!cpu_only)
    {
        TestComposedModelSVGD();
        TestSVGDClassConstantScale();
        for (int w = 0; w < 3; ++w)
            TestSVGDMedianGMM(w);
        TestSVGDMatrixScales(true);
        TestSVGDMatrixScales(false);
    }
    std::printf("%d checks passed, %d failed\n", g_pass, g_fail);
    return g_fail == 0 ? 0 : 1;
}
