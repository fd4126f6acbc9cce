/**
 * @file Adam.hpp
 * @brief Bias-corrected Adam (reference: include/SVGDCpp/Optimizer/Adam.hpp:22-112).
 *
 * m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2;  t++;
 * step = lr * (1 / (eps + sqrt(v / (1-b2^t)))) * (m / (1-b1^t))      (:75-83, :93-96)
 * The device path evaluates the same expression in the same order.
 */
#ifndef SVGDCPP_AMD_ADAM_HPP
#define SVGDCPP_AMD_ADAM_HPP

#include "../Core.hpp"
#include "Optimizer.hpp"

class Adam : public Optimizer
{
public:
    Adam(const size_t &dimension, const size_t &num_particles, const double &lr, const double &beta1,
         const double &beta2, const double &epsilon = 1.0e-8)
        : Optimizer(lr, epsilon), dimension_(dimension), num_particles_(num_particles), decay_rate_1_(beta1),
          decay_rate_2_(beta2)
    {
        if (beta1 >= 1.0 || beta1 < 0.0 || beta2 >= 1.0 || beta2 < 0.0)
            throw std::invalid_argument(SVGDCPP_LOG_PREFIX + "[Argument Error] Invalid value for decay parameter beta.");
    }

    void Initialize() override
    {
        m_ = Eigen::MatrixXd::Zero((long)dimension_, (long)num_particles_);
        v_ = Eigen::MatrixXd::Zero((long)dimension_, (long)num_particles_);
        counter_ = 0;
    }

    Eigen::MatrixXd Step(const Eigen::MatrixXd &g) override
    {
        Eigen::MatrixXd out(g.rows(), g.cols());
        ++counter_;
        const double c1 = 1.0 - std::pow(decay_rate_1_, (double)counter_);
        const double c2 = 1.0 - std::pow(decay_rate_2_, (double)counter_);
        for (long e = 0; e < g.size(); ++e)
        {
            m_(e) = decay_rate_1_ * m_(e) + (1 - decay_rate_1_) * g(e);
            v_(e) = decay_rate_2_ * v_(e) + (1 - decay_rate_2_) * (g(e) * g(e));
            out(e) = (learning_rate_ * (1.0 / (stabilizer_ + std::sqrt(v_(e) / c2)))) * (m_(e) / c1);
        }
        return out;
    }

    int Kind() const override { return SVGD_OPT_ADAM; }
    void Params(double *p) const override
    {
        p[0] = learning_rate_;
        p[1] = decay_rate_1_;
        p[2] = decay_rate_2_;
        p[3] = stabilizer_;
    }

protected:
    size_t counter_ = 0;
    size_t dimension_, num_particles_;
    double decay_rate_1_, decay_rate_2_;
    Eigen::MatrixXd m_, v_;
};

#endif
