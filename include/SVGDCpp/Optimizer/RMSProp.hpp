/**
 * @file RMSProp.hpp
 * @brief RMSProp (reference: include/SVGDCpp/Optimizer/RMSProp.hpp:22-85).
 *
 * v = beta v + (1-beta) g^2;  step = lr * (1 / (eps + sqrt(v))) * g   (:69-74)
 */
#ifndef SVGDCPP_AMD_RMSPROP_HPP
#define SVGDCPP_AMD_RMSPROP_HPP

#include "../Core.hpp"
#include "Optimizer.hpp"

class RMSProp : public Optimizer
{
public:
    RMSProp(const size_t &dimension, const size_t &num_particles, const double &lr, const double &beta,
            const double &epsilon = 1.0e-8)
        : Optimizer(lr, epsilon), dimension_(dimension), num_particles_(num_particles), decay_rate_(beta)
    {
        if (beta > 1.0 || beta < 0.0)
            throw std::invalid_argument(SVGDCPP_LOG_PREFIX + "[Argument Error] Invalid value for decay parameter beta.");
    }

    void Initialize() override { v_ = Eigen::MatrixXd::Zero((long)dimension_, (long)num_particles_); }

    Eigen::MatrixXd Step(const Eigen::MatrixXd &g) override
    {
        Eigen::MatrixXd out(g.rows(), g.cols());
        for (long e = 0; e < g.size(); ++e)
        {
            v_(e) = decay_rate_ * v_(e) + (1 - decay_rate_) * (g(e) * g(e));
            out(e) = (learning_rate_ * (1.0 / (stabilizer_ + std::sqrt(v_(e))))) * g(e);
        }
        return out;
    }

    int Kind() const override { return SVGD_OPT_RMSPROP; }
    void Params(double *p) const override
    {
        p[0] = learning_rate_;
        p[1] = decay_rate_;
        p[2] = 0.0;
        p[3] = stabilizer_;
    }

protected:
    size_t dimension_, num_particles_;
    double decay_rate_;
    Eigen::MatrixXd v_;
};

#endif
