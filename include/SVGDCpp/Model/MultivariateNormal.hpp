/**
 * @file MultivariateNormal.hpp
 * @brief Unnormalised multivariate normal model
 *        (reference: include/SVGDCpp/Model/MultivariateNormal.hpp:23-189).
 *
 * p(x) = exp(-1/2 (x-mu)^T Sigma^-1 (x-mu)) (:56-61), grad log p = -Sigma^-1 (x-mu),
 * evaluated in closed form on the host (CppAD is not part of this build).
 */
#ifndef SVGDCPP_AMD_MULTIVARIATE_NORMAL_HPP
#define SVGDCPP_AMD_MULTIVARIATE_NORMAL_HPP

#include "../Core.hpp"
#include "Model.hpp"

class MultivariateNormal : public Model
{
public:
    MultivariateNormal() {}

    /** :39-64 */
    MultivariateNormal(const Eigen::VectorXd &mean, const Eigen::MatrixXd &covariance) : Model(mean.rows())
    {
        if (!CompareVectorSizes(mean, covariance) || mean.rows() != covariance.cols())
            throw DimensionMismatchException("Dimensions of parameter vectors/matrices do not match.");
        AddGaussian(mean, covariance);
        ComputeNormalizationConstant();
    }

    std::unique_ptr<Model> CloneUniquePointer() const override { return std::make_unique<MultivariateNormal>(*this); }
    std::shared_ptr<Model> CloneSharedPointer() const override { return std::make_shared<MultivariateNormal>(*this); }

    /** :94-115 */
    void UpdateParameters(const std::vector<Eigen::MatrixXd> &params) override
    {
        const Eigen::MatrixXd &mean = params[0];
        const Eigen::MatrixXd &covariance = params[1];
        if (mean.rows() != covariance.rows() || mean.rows() != covariance.cols())
            throw DimensionMismatchException(
                "Dimensions of parameter vectors/matrices do not match each other (# of rows must be equal).");
        else if (mean.rows() != dimension_)
            throw DimensionMismatchException("Dimensions of parameter vectors/matrices do not match original dimension.");
        Model::UpdateParameters(params);
        ComputeNormalizationConstant();
    }

    double EvaluateModelNormalized(const Eigen::VectorXd &x) { return norm_const_ * EvaluateModel(x); }
    double EvaluateLogModelNormalized(const Eigen::VectorXd &x) { return std::log(norm_const_) + EvaluateLogModel(x); }
    double GetNormalizationConstant() { return norm_const_; }

protected:
    /** :182-186 */
    void ComputeNormalizationConstant()
    {
        norm_const_ = 1.0 / (std::pow(2.0 * M_PI, dimension_ / 2.0) * std::sqrt(svgdcpp::Determinant(covs_[0])));
    }

    double norm_const_ = 0.0;
};

#endif
