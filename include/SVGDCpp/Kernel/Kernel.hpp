/**
 * @file Kernel.hpp
 * @brief Kernel plugin base (reference: include/SVGDCpp/Kernel/Kernel.hpp:19-420).
 *
 * In the reference a Kernel is a CppAD-taped function k(x, x') with a
 * "location" x' (the 2nd argument) and parameter matrices.  The SVGD hot path
 * of this build evaluates the Gaussian RBF kernel fused on the device
 * (svgd_phi).  Any other kernel runs on the generic host path of SVGD::Step
 * (SVGD.hpp here), through the same closed-form evaluation virtuals the
 * reference lets a derived kernel override (EvaluateKernel/EvaluateKernelGrad,
 * Kernel.hpp:279-297).
 *
 * CppAD is not part of this build, so a kernel function is set with its
 * gradient in closed form: UpdateKernel(f, grad_f), both taking
 * (x, params, location) like the reference's KernelFun (:391-399).  The
 * reference's functional composition (:55-223: +, -, *, / of two set kernels,
 * parameters concatenated) composes the closed forms with the sum, product and
 * quotient rules.  A kernel with no function and no overrides throws
 * UnsetException on evaluation (:393-396).
 */
#ifndef SVGDCPP_AMD_KERNEL_HPP
#define SVGDCPP_AMD_KERNEL_HPP

#include <functional>

#include "../Core.hpp"

class Kernel
{
public:
    /** k(x, params, location) -- the reference's KernelFun signature over doubles. */
    using KernelFunction =
        std::function<double(const Eigen::VectorXd &, const std::vector<Eigen::MatrixXd> &, const Eigen::VectorXd &)>;
    /** grad_x k(x, params, location), closed form (no tape engine here). */
    using KernelGradFunction = std::function<Eigen::VectorXd(const Eigen::VectorXd &, const std::vector<Eigen::MatrixXd> &,
                                                             const Eigen::VectorXd &)>;

    Kernel() {}
    explicit Kernel(const size_t &dim) : dimension_((int)dim), location_(Eigen::VectorXd::Zero((long)dim)) {}
    virtual ~Kernel() {}

    virtual std::unique_ptr<Kernel> CloneUniquePointer() const { return std::make_unique<Kernel>(*this); }
    virtual std::shared_ptr<Kernel> CloneSharedPointer() const { return std::make_shared<Kernel>(*this); }

    /** Kernel.hpp:55-88: k1 + k2 (parameters of k1 then k2). */
    Kernel operator+(const Kernel &obj) const
    {
        return Compose(obj, [](double a, double b) { return a + b; },
                       [](double, const Eigen::VectorXd &ga, double, const Eigen::VectorXd &gb) { return ga + gb; });
    }

    /** Kernel.hpp:96-129: k1 - k2. */
    Kernel operator-(const Kernel &obj) const
    {
        return Compose(obj, [](double a, double b) { return a - b; },
                       [](double, const Eigen::VectorXd &ga, double, const Eigen::VectorXd &gb) { return ga - gb; });
    }

    /** Kernel.hpp:137-170: k1 * k2 (product rule for the gradient). */
    Kernel operator*(const Kernel &obj) const
    {
        return Compose(obj, [](double a, double b) { return a * b; },
                       [](double a, const Eigen::VectorXd &ga, double b, const Eigen::VectorXd &gb)
                       { return b * ga + a * gb; });
    }

    /** Kernel.hpp:178-223: k1 / k2 (quotient rule for the gradient). */
    Kernel operator/(const Kernel &obj) const
    {
        return Compose(obj, [](double a, double b) { return a / b; },
                       [](double a, const Eigen::VectorXd &ga, double b, const Eigen::VectorXd &gb)
                       { return (b * ga - a * gb) / (b * b); });
    }

    /** Kernel.hpp:264-267 (no tape to record here). */
    virtual void Initialize() {}

    /** k(x, location) (Kernel.hpp:279): the set function, or a derived override. */
    virtual double EvaluateKernel(const Eigen::VectorXd &x)
    {
        if (!kernel_fun_)
            throw UnsetException("Kernel function is unset.");
        return kernel_fun_(x, kernel_parameters_, location_);
    }

    /** grad_x k(x, location) (Kernel.hpp:294). */
    virtual Eigen::VectorXd EvaluateKernelGrad(const Eigen::VectorXd &x)
    {
        if (!kernel_grad_fun_)
            throw UnsetException("Kernel function is unset.");
        return kernel_grad_fun_(x, kernel_parameters_, location_);
    }

    /** Kernel.hpp:304-315 */
    virtual void UpdateParameters(const std::vector<Eigen::MatrixXd> &params) { kernel_parameters_ = params; }

    /** Kernel.hpp:322-330 */
    virtual void UpdateLocation(const Eigen::VectorXd &x)
    {
        if (x.rows() != dimension_)
            throw DimensionMismatchException("Dimension mismatch between provided location and kernel dimension (" +
                                             std::to_string(x.rows()) + " vs. " + std::to_string(dimension_) + ").");
        location_ = x;
    }

    std::vector<Eigen::MatrixXd> GetParameters() const { return kernel_parameters_; }

    /** Kernel.hpp:356: per-step hook. */
    virtual void Step() {}

    /** Kernel.hpp:365-368, with the gradient in closed form. */
    void UpdateKernel(KernelFunction kernel_fun, KernelGradFunction kernel_grad_fun)
    {
        kernel_fun_ = std::move(kernel_fun);
        kernel_grad_fun_ = std::move(kernel_grad_fun);
    }

    int GetDimension() const { return dimension_; }

protected:
    template <class F, class G> Kernel Compose(const Kernel &obj, F f, G g) const
    {
        if (dimension_ != obj.dimension_)
            throw DimensionMismatchException("Only kernels with the same variable dimensions can be added.");
        if (!kernel_fun_ || !obj.kernel_fun_ || !kernel_grad_fun_ || !obj.kernel_grad_fun_)
            throw UnsetException("One of the kernel functions is unset; functional composition requires both kernel "
                                 "functions to be set.");
        Kernel out((size_t)dimension_);
        out.kernel_parameters_ = kernel_parameters_;
        out.kernel_parameters_.insert(out.kernel_parameters_.end(), obj.kernel_parameters_.begin(),
                                      obj.kernel_parameters_.end());
        // copies of both operands' functions (the reference captures the
        // operands by reference, which dangles once they go out of scope)
        const size_t n1 = kernel_parameters_.size();
        auto split = [n1](const std::vector<Eigen::MatrixXd> &p) {
            return std::make_pair(std::vector<Eigen::MatrixXd>(p.begin(), p.begin() + (long)n1),
                                  std::vector<Eigen::MatrixXd>(p.begin() + (long)n1, p.end()));
        };
        const KernelFunction f1 = kernel_fun_, f2 = obj.kernel_fun_;
        const KernelGradFunction g1 = kernel_grad_fun_, g2 = obj.kernel_grad_fun_;
        out.kernel_fun_ = [=](const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &p,
                              const Eigen::VectorXd &loc) {
            const auto pp = split(p);
            return f(f1(x, pp.first, loc), f2(x, pp.second, loc));
        };
        out.kernel_grad_fun_ = [=](const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &p,
                                   const Eigen::VectorXd &loc) {
            const auto pp = split(p);
            return Eigen::VectorXd(g(f1(x, pp.first, loc), g1(x, pp.first, loc), f2(x, pp.second, loc),
                                     g2(x, pp.second, loc)));
        };
        return out;
    }

    int dimension_ = -1;
    Eigen::VectorXd location_;
    std::vector<Eigen::MatrixXd> kernel_parameters_;
    KernelFunction kernel_fun_;
    KernelGradFunction kernel_grad_fun_;
};

#endif
