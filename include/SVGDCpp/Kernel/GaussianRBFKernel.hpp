/**
 * @file GaussianRBFKernel.hpp
 * @brief Gaussian RBF kernel (reference: include/SVGDCpp/Kernel/GaussianRBFKernel.hpp:22-270).
 *
 * k(x, x') = exp(-(x - x')^T M (x - x')) (:75-81).
 *   ScaleMethod::Median   M = a I, a = ln(N) / med^2, med = median of all N^2
 *                         pairwise distances of the coordinate matrix (:168-188)
 *                         -- recomputed every step ON THE DEVICE by the SVGD driver.
 *   ScaleMethod::Hessian  M = sum_i -hess log p(x_i) / (2 d N) (:189-210) --
 *                         the model's Hessians summed on the host, M and its
 *                         Cholesky factor formed on the device each step.
 *   ScaleMethod::Constant extension (the reference's "TODO: constant scale"):
 *                         a fixed M set by UpdateParameters({M}), isotropic
 *                         a I or any symmetric positive-definite matrix.
 * The host methods below (ComputeScale, EvaluateKernel/Grad) restate the
 * kernel for callers that use it directly; SVGD does not call them.
 */
#ifndef SVGDCPP_AMD_GAUSSIAN_RBF_KERNEL_HPP
#define SVGDCPP_AMD_GAUSSIAN_RBF_KERNEL_HPP

#include "../Core.hpp"
#include "../Model/Model.hpp"
#include "Kernel.hpp"

class GaussianRBFKernel : public Kernel
{
public:
    enum class ScaleMethod
    {
        Median = 0,
        Hessian = 1,
        Constant = 2
    };

    GaussianRBFKernel() {}

    /** :47-88 */
    GaussianRBFKernel(const std::shared_ptr<Eigen::MatrixXd> &coord_mat_ptr, const ScaleMethod &method = ScaleMethod::Median,
                      const std::shared_ptr<Model> &model_ptr = nullptr)
        : Kernel((size_t)coord_mat_ptr->rows()), scale_method_(method), coord_matrix_ptr_(coord_mat_ptr),
          target_model_ptr_(model_ptr)
    {
        if (scale_method_ == ScaleMethod::Hessian && !model_ptr) // :55-58
            throw UnsetException("Hessian-based scale requires a model.");
        // The reference computes the median scale here (:84) and again in every
        // Step() before it is used (SVGD.hpp:389); the device recomputes it per
        // step, so no O(N^2) host work happens at construction.
        kernel_parameters_ = {Eigen::MatrixXd::Identity(dimension_, dimension_)};
        // the closed form as the kernel function too (the reference sets its
        // lambda with UpdateKernel, :75-87), so rbf + k, rbf * k, ... compose
        // on the generic host path like any other set kernel
        UpdateKernel(&GaussianRBFKernel::Value, &GaussianRBFKernel::Grad);
    }

    /** :75-81 -- exp(-(x - loc)^T M (x - loc)), M = params[0]. */
    static double Value(const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &params,
                        const Eigen::VectorXd &loc)
    {
        const Eigen::MatrixXd &M = params.at(0);
        const long d = x.rows();
        double s = 0.0;
        for (long r = 0; r < d; ++r)
        {
            double t = 0.0;
            for (long c = 0; c < d; ++c)
                t += M(r, c) * (x(c) - loc(c));
            s += (x(r) - loc(r)) * t;
        }
        return std::exp(-s);
    }

    /** grad_x: -2 M (x - loc) k(x, loc) (the reference's CppAD Jacobian of :75-81). */
    static Eigen::VectorXd Grad(const Eigen::VectorXd &x, const std::vector<Eigen::MatrixXd> &params,
                                const Eigen::VectorXd &loc)
    {
        const Eigen::MatrixXd &M = params.at(0);
        const long d = x.rows();
        const double kv = Value(x, params, loc);
        Eigen::VectorXd g(d);
        for (long r = 0; r < d; ++r)
        {
            double t = 0.0;
            for (long c = 0; c < d; ++c)
                t += M(r, c) * (x(c) - loc(c));
            g(r) = -2.0 * t * kv;
        }
        return g;
    }

    std::unique_ptr<Kernel> CloneUniquePointer() const override { return std::make_unique<GaussianRBFKernel>(*this); }
    std::shared_ptr<Kernel> CloneSharedPointer() const override { return std::make_shared<GaussianRBFKernel>(*this); }

    ScaleMethod GetScaleMethod() const { return scale_method_; }
    std::shared_ptr<Model> GetTargetModel() const { return target_model_ptr_; }

    /** The scale matrix M (kernel_parameters_[0]). */
    const Eigen::MatrixXd &GetScaleMatrix() const { return kernel_parameters_.at(0); }

    /** a of M = a I (M(0,0) for a full matrix). */
    double GetScale() const { return GetScaleMatrix()(0, 0); }

    /** True when M = a I. */
    bool IsIsotropic() const
    {
        const Eigen::MatrixXd &M = GetScaleMatrix();
        for (long r = 0; r < M.rows(); ++r)
            for (long c = 0; c < M.cols(); ++c)
                if (M(r, c) != (r == c ? M(0, 0) : 0.0))
                    return false;
        return true;
    }

    void UpdateParameters(const std::vector<Eigen::MatrixXd> &params) override
    {
        const Eigen::MatrixXd &M = params.at(0);
        if (M.rows() != dimension_ || M.cols() != dimension_)
            throw DimensionMismatchException("Kernel scale matrix has incorrect dimensions.");
        kernel_parameters_ = {M};
    }

    /** exp(-(x - location)^T M (x - location)) */
    double EvaluateKernel(const Eigen::VectorXd &x) override { return Value(x, kernel_parameters_, location_); }

    /** -2 M (x - location) k(x, location) */
    Eigen::VectorXd EvaluateKernelGrad(const Eigen::VectorXd &x) override
    {
        return Grad(x, kernel_parameters_, location_);
    }

    /** :141-156 -- host restatement; the SVGD driver computes the scale on the device. */
    void Step() override
    {
        if (scale_method_ != ScaleMethod::Constant)
            kernel_parameters_[0] = ComputeScale();
    }

    /** :164-210 on the host: the median heuristic (O(N^2) memory, small N
     *  only) or the Hessian heuristic. */
    Eigen::MatrixXd ComputeScale()
    {
        const Eigen::MatrixXd &X = *coord_matrix_ptr_;
        if (scale_method_ == ScaleMethod::Hessian)
        {
            const long n = X.cols(), d = X.rows();
            Eigen::MatrixXd H(d, d), M(d, d);
            std::vector<double> rows((size_t)(n * d)), Hs((size_t)(d * d));
            std::copy(X.data(), X.data() + n * d, rows.data());
            target_model_ptr_->NegHessSumBatch(rows.data(), n, Hs.data());
            for (long r = 0; r < d; ++r)
                for (long c = 0; c < d; ++c)
                    M(r, c) = Hs[(size_t)(r * d + c)] / (2.0 * (double)d * (double)n);
            return M;
        }
        const long n = X.cols(), d = X.rows();
        std::vector<double> dist((size_t)(n * n));
        for (long j = 0; j < n; ++j)
            for (long i = 0; i < n; ++i)
            {
                double s = 0.0;
                for (long k = 0; k < d; ++k)
                    s += (X(k, i) - X(k, j)) * (X(k, i) - X(k, j));
                dist[(size_t)(j * n + i)] = std::sqrt(s);
            }
        const size_t h = dist.size() / 2;
        std::nth_element(dist.begin(), dist.begin() + (long)h, dist.end());
        double med = dist[h];
        if (dist.size() % 2 == 0)
            med = (med + *std::max_element(dist.begin(), dist.begin() + (long)h)) / 2.0;
        return std::log((double)n) / std::pow(med, 2) * Eigen::MatrixXd::Identity(d, d);
    }

protected:
    ScaleMethod scale_method_ = ScaleMethod::Median;
    std::shared_ptr<Eigen::MatrixXd> coord_matrix_ptr_;
    std::shared_ptr<Model> target_model_ptr_;
};

#endif
