/**
 * @file Model.hpp
 * @brief Target density plugin (reference: include/SVGDCpp/Model/Model.hpp:20-494).
 *
 * The model's log-gradient stays on the host (the reference evaluates
 * EvaluateLogModelGrad per particle, SVGD.hpp:438).  CppAD is not part of
 * this build, so a user model overrides the closed forms -- the reference's
 * documented "Method 3" (doc/instructions.md:234-301):
 *
 *   class MyModel : public Model {
 *       Eigen::VectorXd EvaluateLogModelGrad(const Eigen::VectorXd &x) override;
 *   };
 *
 * Built-in Gaussian models (MultivariateNormal and their operator+ sums, the
 * reference's Model.hpp:55-92 composition) evaluate all particles at once in
 * C++ with OpenMP through svgd_model_logp_grad.
 */
#ifndef SVGDCPP_AMD_MODEL_HPP
#define SVGDCPP_AMD_MODEL_HPP

#include "../Core.hpp"

class Model
{
public:
    Model() {}
    explicit Model(const size_t &dim) : dimension_((int)dim) {}
    Model(const Model &o) { *this = o; }
    Model &operator=(const Model &o)
    {
        dimension_ = o.dimension_;
        means_ = o.means_;
        covs_ = o.covs_;
        handle_.reset();
        return *this;
    }
    virtual ~Model() {}

    /** Model.hpp:55-92: the density of the sum is the sum of the densities
     *  (unweighted, unnormalised).  Supported for Gaussian-sum models. */
    Model operator+(const Model &obj) const
    {
        if (dimension_ != obj.dimension_)
            throw DimensionMismatchException("Only models with the same variable dimensions can be added.");
        if (means_.empty() || obj.means_.empty())
            throw UnsetException("One of the model functions is unset; functional composition requires both "
                                 "model functions to be set.");
        Model m((size_t)dimension_);
        m.means_ = means_;
        m.covs_ = covs_;
        m.means_.insert(m.means_.end(), obj.means_.begin(), obj.means_.end());
        m.covs_.insert(m.covs_.end(), obj.covs_.begin(), obj.covs_.end());
        return m;
    }

    virtual std::unique_ptr<Model> CloneUniquePointer() const { return std::make_unique<Model>(*this); }
    virtual std::shared_ptr<Model> CloneSharedPointer() const { return std::make_shared<Model>(*this); }

    /** Model.hpp:268-278. */
    virtual void Initialize()
    {
        if (dimension_ <= 0)
            throw UnsetException("Model dimension (" + std::to_string(dimension_) + ") is improperly or not set.");
        if (!means_.empty())
            Build();
    }

    /** Model.hpp:413: per-step hook (no-op by default). */
    virtual void Step() {}

    /** Unnormalised density (Model.hpp:290). */
    virtual double EvaluateModel(const Eigen::VectorXd &x) { return std::exp(EvaluateLogModel(x)); }

    /** log density (Model.hpp:305), log-sum-exp over the Gaussian terms. */
    virtual double EvaluateLogModel(const Eigen::VectorXd &x)
    {
        RequireGaussian();
        double qmin = INFINITY;
        std::vector<double> q(means_.size());
        for (size_t c = 0; c < means_.size(); ++c)
        {
            Eigen::VectorXd diff = x - means_[c];
            Eigen::MatrixXd P = svgdcpp::Inverse(covs_[c]);
            q[c] = 0.5 * (diff.transpose() * (P * diff))(0, 0);
            qmin = std::min(qmin, q[c]);
        }
        double s = 0.0;
        for (double v : q)
            s += std::exp(-(v - qmin));
        return -qmin + std::log(s);
    }

    /** grad log p at one particle (Model.hpp:335-338). */
    virtual Eigen::VectorXd EvaluateLogModelGrad(const Eigen::VectorXd &x)
    {
        RequireGaussian();
        Eigen::VectorXd g(dimension_);
        LogModelGradBatch(x.data(), 1, g.data());
        return g;
    }

    /**
     * grad log p for n particles (rows of X, particle i at X + i*d) -- the
     * call the SVGD driver makes once per step.  Gaussian models use the C++
     * host kernel; other models fall back to EvaluateLogModelGrad per
     * particle, serially, as the reference does (SVGD.hpp:412-416).
     */
    virtual void LogModelGradBatch(const double *X, int64_t n, double *G)
    {
        if (!means_.empty())
        {
            if (!handle_)
                Build();
            const int rc = svgd_model_logp_grad(handle_.get(), X, n, G);
            if (rc != SVGD_OK)
                svgdcpp::ThrowFromCode(rc, SVGDCPP_LOG_PREFIX + "[Runtime Error] host model evaluation failed.");
            return;
        }
        Eigen::VectorXd x(dimension_);
        for (int64_t i = 0; i < n; ++i)
        {
            std::copy(X + i * dimension_, X + (i + 1) * dimension_, x.data());
            Eigen::VectorXd g = EvaluateLogModelGrad(x);
            if (g.rows() != dimension_)
                throw DimensionMismatchException("EvaluateLogModelGrad returned a vector of the wrong size.");
            std::copy(g.data(), g.data() + dimension_, G + i * dimension_);
        }
    }

    /** hess log p at one particle (Model.hpp:366-370).  Gaussian models use
     *  the closed form; other models override it to use the Hessian scale. */
    virtual Eigen::MatrixXd EvaluateLogModelHessian(const Eigen::VectorXd &x)
    {
        RequireGaussian();
        Eigen::MatrixXd H((long)dimension_, (long)dimension_);
        NegHessSumBatch(x.data(), 1, H.data());
        for (long e = 0; e < H.size(); ++e)
            H(e) = -H(e);
        return H;
    }

    /**
     * sum_i -hess log p(x_i) over n particles (row-major d x d; symmetric) --
     * the sum inside the Hessian kernel scale (GaussianRBFKernel.hpp:197-205).
     */
    virtual void NegHessSumBatch(const double *X, int64_t n, double *H)
    {
        const long d = dimension_;
        if (!means_.empty())
        {
            if (!handle_)
                Build();
            const int rc = svgd_model_neg_hess_sum(handle_.get(), X, n, H);
            if (rc != SVGD_OK)
                svgdcpp::ThrowFromCode(rc, SVGDCPP_LOG_PREFIX + "[Runtime Error] host model evaluation failed.");
            return;
        }
        std::fill(H, H + d * d, 0.0);
        Eigen::VectorXd x(d);
        for (int64_t i = 0; i < n; ++i)
        {
            std::copy(X + i * d, X + (i + 1) * d, x.data());
            const Eigen::MatrixXd h = EvaluateLogModelHessian(x);
            for (long r = 0; r < d; ++r)
                for (long c = 0; c < d; ++c)
                    H[r * d + c] -= h(r, c);
        }
    }

    /** Model.hpp:377-388: replace the parameter matrices (Gaussian terms: mean0, cov0, mean1, cov1, ...). */
    virtual void UpdateParameters(const std::vector<Eigen::MatrixXd> &params)
    {
        if (params.size() != 2 * means_.size())
            throw DimensionMismatchException("Number of parameters does not match the model.");
        for (size_t c = 0; c < means_.size(); ++c)
        {
            means_[c] = Eigen::VectorXd(params[2 * c]);
            covs_[c] = params[2 * c + 1];
        }
        handle_.reset();
    }

    /** Model.hpp:395-406. */
    std::vector<Eigen::MatrixXd> GetParameters() const
    {
        std::vector<Eigen::MatrixXd> p;
        for (size_t c = 0; c < means_.size(); ++c)
        {
            p.push_back(means_[c]);
            p.push_back(covs_[c]);
        }
        return p;
    }

    int GetDimension() const { return dimension_; }

protected:
    void AddGaussian(const Eigen::VectorXd &mean, const Eigen::MatrixXd &cov)
    {
        means_.push_back(mean);
        covs_.push_back(cov);
        handle_.reset();
    }
    void RequireGaussian() const
    {
        if (means_.empty())
            throw UnsetException("Model function is unset.");
    }
    void Build()
    {
        const int d = dimension_, k = (int)means_.size();
        std::vector<double> mus((size_t)k * d), covs((size_t)k * d * d);
        for (int c = 0; c < k; ++c)
            for (int r = 0; r < d; ++r)
            {
                mus[(size_t)c * d + r] = means_[c](r);
                for (int l = 0; l < d; ++l)
                    covs[((size_t)c * d + r) * d + l] = covs_[c](r, l);
            }
        void *h = nullptr;
        const int rc = svgd_model_create(&h, d, k, mus.data(), covs.data());
        if (rc != SVGD_OK)
            svgdcpp::ThrowFromCode(rc, SVGDCPP_LOG_PREFIX + "[Argument Error] Singular covariance matrix.");
        handle_.reset(h, [](void *p) { svgd_model_destroy(p); });
    }

    int dimension_ = -1;
    std::vector<Eigen::VectorXd> means_;
    std::vector<Eigen::MatrixXd> covs_;
    std::shared_ptr<void> handle_;
};

#endif
