/**
 * @file Kernel.hpp
 * @brief Kernel plugin base (reference: include/SVGDCpp/Kernel/Kernel.hpp:19-420).
 *
 * In the reference a Kernel is a CppAD-taped function k(x, x') with a
 * "location" x' (the 2nd argument) and parameter matrices.  The SVGD hot path
 * of this build only evaluates the Gaussian RBF kernel, fused on the device
 * (svgd_phi), so the base class keeps the plugin contract -- dimension,
 * location, parameters, per-step hook -- and the closed-form evaluation
 * virtuals that derived kernels override (EvaluateKernel/EvaluateKernelGrad,
 * Kernel.hpp:279-297).
 */
#ifndef SVGDCPP_AMD_KERNEL_HPP
#define SVGDCPP_AMD_KERNEL_HPP

#include "../Core.hpp"

class Kernel
{
public:
    Kernel() {}
    explicit Kernel(const size_t &dim) : dimension_((int)dim), location_(Eigen::VectorXd::Zero((long)dim)) {}
    virtual ~Kernel() {}

    virtual std::unique_ptr<Kernel> CloneUniquePointer() const { return std::make_unique<Kernel>(*this); }
    virtual std::shared_ptr<Kernel> CloneSharedPointer() const { return std::make_shared<Kernel>(*this); }

    /** Kernel.hpp:264-267 (no tape to record here). */
    virtual void Initialize() {}

    /** k(x, location) -- override in derived kernels (Kernel.hpp:279). */
    virtual double EvaluateKernel(const Eigen::VectorXd &) { throw UnsetException("Kernel function is unset."); }

    /** grad_x k(x, location) (Kernel.hpp:294). */
    virtual Eigen::VectorXd EvaluateKernelGrad(const Eigen::VectorXd &)
    {
        throw UnsetException("Kernel function is unset.");
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

    int GetDimension() const { return dimension_; }

protected:
    int dimension_ = -1;
    Eigen::VectorXd location_;
    std::vector<Eigen::MatrixXd> kernel_parameters_;
};

#endif
