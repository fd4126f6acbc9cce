/**
 * @file Optimizer.hpp
 * @brief Optimizer plugin base (reference: include/SVGDCpp/Optimizer/Optimizer.hpp:19-48).
 *
 * Contract kept: Initialize() resets state, Step(grad) returns the increment
 * that the driver adds to the coordinates (SVGD.hpp:393).  The built-in
 * optimizers also describe themselves to the device path (Kind/Params), where
 * the same element-wise update runs fused with the clamp.
 */
#ifndef SVGDCPP_AMD_OPTIMIZER_HPP
#define SVGDCPP_AMD_OPTIMIZER_HPP

#include "../Core.hpp"

class Optimizer
{
public:
    Optimizer(const double &lr, const double &epsilon = 1.0e-8) : learning_rate_(lr), stabilizer_(epsilon) {}
    virtual ~Optimizer() {}

    virtual void Initialize() = 0;
    virtual Eigen::MatrixXd Step(const Eigen::MatrixXd &grad_matrix) = 0;

    /** Device kind (SVGD_OPT_*) or -1 for optimizers without a device kernel. */
    virtual int Kind() const { return -1; }
    /** lr, beta1 (or beta), beta2, eps for svgd_set_optimizer. */
    virtual void Params(double *p) const
    {
        p[0] = learning_rate_;
        p[1] = p[2] = 0.0;
        p[3] = stabilizer_;
    }

protected:
    double learning_rate_;
    double stabilizer_;
};

#endif
