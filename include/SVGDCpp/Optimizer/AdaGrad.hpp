/**
 * @file AdaGrad.hpp
 * @brief AdaGrad (reference: include/SVGDCpp/Optimizer/AdaGrad.hpp:22-76).
 *
 * v += g^2;  step = lr * (1 / (eps + sqrt(v))) * g     (:60-65)
 */
#ifndef SVGDCPP_AMD_ADAGRAD_HPP
#define SVGDCPP_AMD_ADAGRAD_HPP

#include "../Core.hpp"
#include "Optimizer.hpp"

class AdaGrad : public Optimizer
{
public:
    AdaGrad(const size_t &dimension, const size_t &num_particles, const double &lr, const double &epsilon = 1.0e-8)
        : Optimizer(lr, epsilon), dimension_(dimension), num_particles_(num_particles)
    {
    }

    void Initialize() override { v_ = Eigen::MatrixXd::Zero((long)dimension_, (long)num_particles_); }

    Eigen::MatrixXd Step(const Eigen::MatrixXd &g) override
    {
        Eigen::MatrixXd out(g.rows(), g.cols());
        for (long e = 0; e < g.size(); ++e)
        {
            v_(e) += g(e) * g(e);
            out(e) = (learning_rate_ * (1.0 / (stabilizer_ + std::sqrt(v_(e))))) * g(e);
        }
        return out;
    }

    int Kind() const override { return SVGD_OPT_ADAGRAD; }

protected:
    size_t dimension_, num_particles_;
    double decay_rate_ = 0.0; ///< unused, as in the reference (:72)
    Eigen::MatrixXd v_;
};

#endif
