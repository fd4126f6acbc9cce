/**
 * @file Model.hpp
 * @brief Target density plugin (reference: include/SVGDCpp/Model/Model.hpp:20-494).
 *
 * The model's log-gradient stays on the host (the reference evaluates
 * EvaluateLogModelGrad per particle, SVGD.hpp:438).  CppAD is not part of
 * this build, so a model is given in closed form -- the reference's
 * documented "Method 3" (doc/instructions.md:234-301) -- either by
 * overriding the evaluation virtuals:
 *
 *   class MyModel : public Model {
 *       double EvaluateModel(const Eigen::VectorXd &x) override;
 *       Eigen::VectorXd EvaluateModelGrad(const Eigen::VectorXd &x) override;
 *       std::shared_ptr<Model> CloneSharedPointer() const override;  // to compose
 *   };
 *
 * or by setting the function with its derivatives, UpdateModel(f, grad_f
 * [, hess_f]), each taking (x, params) like the reference's ModelFun
 * (:434-443).  The composition operators + - * / (:55-227) compose the
 * closed forms with the sum, product and quotient rules (value, gradient,
 * Hessian) over copies of the operands (CloneSharedPointer: a derived model
 * that overrides the virtuals overrides it too, as MultivariateNormal
 * does; the reference captures the operands by reference, which dangles once
 * they go out of scope); log p, grad log p and hess log p of a composed or
 * function model follow from them (grad log p = grad p / p,
 * hess log p = hess p / p - grad p grad p^T / p^2), as the reference's
 * LogModelFun (:451-454) differentiates log(ModelFun).
 *
 * Built-in Gaussian models (MultivariateNormal and their operator+ sums, the
 * reference's Model.hpp:55-92 composition with unweighted, unnormalised
 * terms) keep their fast path: a sum of Gaussian forms stays a Gaussian
 * form, and all particles are evaluated at once in C++ with OpenMP through
 * svgd_model_logp_grad.
 */
#ifndef SVGDCPP_AMD_MODEL_HPP
#define SVGDCPP_AMD_MODEL_HPP

#include <functional>
#include <typeinfo>

#include "../Core.hpp"

class Model
{
public:
    /** p(x, params) -- the reference's ModelFun signature over doubles. */
    using ModelFunction = std::function<double(const Eigen::VectorXd &, const std::vector<Eigen::MatrixXd> &)>;
    /** grad_x p(x, params), closed form (no tape engine here). */
    using ModelGradFunction =
        std::function<Eigen::VectorXd(const Eigen::VectorXd &, const std::vector<Eigen::MatrixXd> &)>;
    /** hess_x p(x, params), closed form (optional: the Hessian kernel scale). */
    using ModelHessFunction =
        std::function<Eigen::MatrixXd(const Eigen::VectorXd &, const std::vector<Eigen::MatrixXd> &)>;

    Model() {}
    explicit Model(const size_t &dim) : dimension_((int)dim) {}
    Model(const Model &o) { *this = o; }
    Model &operator=(const Model &o)
    {
        dimension_ = o.dimension_;
        means_ = o.means_;
        covs_ = o.covs_;
        model_parameters_ = o.model_parameters_;
        model_fun_ = o.model_fun_;
        model_grad_fun_ = o.model_grad_fun_;
        model_hess_fun_ = o.model_hess_fun_;
        op_ = o.op_;
        lhs_ = o.lhs_;
        rhs_ = o.rhs_;
        handle_.reset();
        return *this;
    }
    virtual ~Model() {}

    /** Model.hpp:55-92: p1 + p2.  Two Gaussian forms (MultivariateNormal and
     *  their sums) give a Gaussian form (unweighted, unnormalised terms:
     *  the host fast path); otherwise the closed forms compose. */
    Model operator+(const Model &obj) const
    {
        CheckComposable(obj, "added");
        if (IsGaussianForm() && obj.IsGaussianForm())
        {
            Model m((size_t)dimension_);
            m.means_ = means_;
            m.covs_ = covs_;
            m.means_.insert(m.means_.end(), obj.means_.begin(), obj.means_.end());
            m.covs_.insert(m.covs_.end(), obj.covs_.begin(), obj.covs_.end());
            return m;
        }
        return Composed(obj, '+');
    }

    /** Model.hpp:100-137: p1 - p2. */
    Model operator-(const Model &obj) const
    {
        CheckComposable(obj, "added");
        return Composed(obj, '-');
    }

    /** Model.hpp:145-182: p1 * p2 (product rule). */
    Model operator*(const Model &obj) const
    {
        CheckComposable(obj, "multiplied");
        return Composed(obj, '*');
    }

    /** Model.hpp:190-227: p1 / p2 (quotient rule). */
    Model operator/(const Model &obj) const
    {
        CheckComposable(obj, "multiplied");
        return Composed(obj, '/');
    }

    virtual std::unique_ptr<Model> CloneUniquePointer() const { return std::make_unique<Model>(*this); }
    virtual std::shared_ptr<Model> CloneSharedPointer() const { return std::make_shared<Model>(*this); }

    /** Model.hpp:268-278. */
    virtual void Initialize()
    {
        if (dimension_ <= 0)
            throw UnsetException("Model dimension (" + std::to_string(dimension_) + ") is improperly or not set.");
        if (IsGaussianForm())
            Build();
        if (lhs_)
        {
            lhs_->Initialize();
            rhs_->Initialize();
        }
    }

    /** Model.hpp:413: per-step hook (no-op by default). */
    virtual void Step() {}

    /** Unnormalised density (Model.hpp:290). */
    virtual double EvaluateModel(const Eigen::VectorXd &x)
    {
        if (model_fun_)
            return model_fun_(x, model_parameters_);
        if (lhs_)
            return Combine(lhs_->EvaluateModel(x), rhs_->EvaluateModel(x));
        if (IsGaussianForm())
            return std::exp(EvaluateLogModel(x));
        throw UnsetException("Model function is unset.");
    }

    /** log density (Model.hpp:305): log-sum-exp over Gaussian terms, else log p. */
    virtual double EvaluateLogModel(const Eigen::VectorXd &x)
    {
        if (IsGaussianForm())
        {
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
        return std::log(EvaluateModel(x));
    }

    /** grad p (Model.hpp:320). */
    virtual Eigen::VectorXd EvaluateModelGrad(const Eigen::VectorXd &x)
    {
        if (model_grad_fun_)
            return model_grad_fun_(x, model_parameters_);
        if (lhs_)
        {
            const double a = lhs_->EvaluateModel(x), b = rhs_->EvaluateModel(x);
            const Eigen::VectorXd ga = lhs_->EvaluateModelGrad(x), gb = rhs_->EvaluateModelGrad(x);
            switch (op_)
            {
            case '+': return ga + gb;
            case '-': return ga - gb;
            case '*': return b * ga + a * gb;
            default: return (b * ga - a * gb) / (b * b);
            }
        }
        if (IsGaussianForm())
            return EvaluateModel(x) * EvaluateLogModelGrad(x);
        throw UnsetException("Model function is unset.");
    }

    /** grad log p at one particle (Model.hpp:335-338). */
    virtual Eigen::VectorXd EvaluateLogModelGrad(const Eigen::VectorXd &x)
    {
        if (IsGaussianForm())
        {
            Eigen::VectorXd g(dimension_);
            LogModelGradBatch(x.data(), 1, g.data());
            return g;
        }
        return EvaluateModelGrad(x) / EvaluateModel(x);
    }

    /** hess p (Model.hpp:350). */
    virtual Eigen::MatrixXd EvaluateModelHessian(const Eigen::VectorXd &x)
    {
        if (model_hess_fun_)
            return model_hess_fun_(x, model_parameters_);
        if (lhs_)
        {
            const double a = lhs_->EvaluateModel(x), b = rhs_->EvaluateModel(x);
            const Eigen::VectorXd ga = lhs_->EvaluateModelGrad(x), gb = rhs_->EvaluateModelGrad(x);
            const Eigen::MatrixXd Ha = lhs_->EvaluateModelHessian(x), Hb = rhs_->EvaluateModelHessian(x);
            const Eigen::MatrixXd cross = ga * gb.transpose() + gb * ga.transpose();
            switch (op_)
            {
            case '+': return Ha + Hb;
            case '-': return Ha - Hb;
            case '*': return b * Ha + cross + a * Hb;
            default: // (a/b)'' = a''/b - (a'b'^T + b'a'^T)/b^2 + 2a b'b'^T/b^3 - a b''/b^2
                return Ha / b - cross / (b * b) + (2.0 * a / (b * b * b)) * (gb * gb.transpose()) -
                       (a / (b * b)) * Hb;
            }
        }
        if (IsGaussianForm())
        {
            const Eigen::VectorXd g = EvaluateLogModelGrad(x);
            return EvaluateModel(x) * (EvaluateLogModelHessian(x) + g * g.transpose());
        }
        throw UnsetException("Model function is unset.");
    }

    /**
     * grad log p for n particles (rows of X, particle i at X + i*d) -- the
     * call the SVGD driver makes once per step.  Gaussian forms use the C++
     * host kernel; other models EvaluateLogModelGrad per particle, serially,
     * as the reference does (SVGD.hpp:412-416).
     */
    virtual void LogModelGradBatch(const double *X, int64_t n, double *G)
    {
        if (IsGaussianForm())
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

    /** hess log p at one particle (Model.hpp:366-370): the Gaussian closed
     *  form, else hess p / p - grad p grad p^T / p^2. */
    virtual Eigen::MatrixXd EvaluateLogModelHessian(const Eigen::VectorXd &x)
    {
        if (IsGaussianForm())
        {
            Eigen::MatrixXd H((long)dimension_, (long)dimension_);
            NegHessSumBatch(x.data(), 1, H.data());
            for (long e = 0; e < H.size(); ++e)
                H(e) = -H(e);
            return H;
        }
        const double p = EvaluateModel(x);
        const Eigen::VectorXd g = EvaluateModelGrad(x);
        return EvaluateModelHessian(x) / p - (g * g.transpose()) / (p * p);
    }

    /**
     * sum_i -hess log p(x_i) over n particles (row-major d x d; symmetric) --
     * the sum inside the Hessian kernel scale (GaussianRBFKernel.hpp:197-205).
     */
    virtual void NegHessSumBatch(const double *X, int64_t n, double *H)
    {
        const long d = dimension_;
        if (IsGaussianForm())
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

    /** Model.hpp:377-388: replace the parameter matrices -- Gaussian terms:
     *  mean0, cov0, mean1, cov1, ...; a composed model: the left operand's
     *  then the right operand's (the reference's concatenation, :70-74). */
    virtual void UpdateParameters(const std::vector<Eigen::MatrixXd> &params)
    {
        if (lhs_)
        {
            const size_t n1 = lhs_->GetParameters().size();
            if (params.size() != n1 + rhs_->GetParameters().size())
                throw DimensionMismatchException("Number of parameters does not match the model.");
            // copy on write: copies of this model share the operands
            lhs_ = lhs_->CloneSharedPointer();
            rhs_ = rhs_->CloneSharedPointer();
            lhs_->UpdateParameters(std::vector<Eigen::MatrixXd>(params.begin(), params.begin() + (long)n1));
            rhs_->UpdateParameters(std::vector<Eigen::MatrixXd>(params.begin() + (long)n1, params.end()));
            return;
        }
        if (!IsGaussianForm())
        {
            model_parameters_ = params;
            return;
        }
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
        if (lhs_)
        {
            std::vector<Eigen::MatrixXd> p = lhs_->GetParameters(), q = rhs_->GetParameters();
            p.insert(p.end(), q.begin(), q.end());
            return p;
        }
        if (!IsGaussianForm())
            return model_parameters_;
        std::vector<Eigen::MatrixXd> p;
        for (size_t c = 0; c < means_.size(); ++c)
        {
            p.push_back(means_[c]);
            p.push_back(covs_[c]);
        }
        return p;
    }

    /** Model.hpp:421-424, with the derivatives in closed form. */
    void UpdateModel(ModelFunction model_fun, ModelGradFunction model_grad_fun,
                     ModelHessFunction model_hess_fun = nullptr)
    {
        model_fun_ = std::move(model_fun);
        model_grad_fun_ = std::move(model_grad_fun);
        model_hess_fun_ = std::move(model_hess_fun);
        means_.clear();
        covs_.clear();
        lhs_.reset();
        rhs_.reset();
        handle_.reset();
    }

    int GetDimension() const { return dimension_; }

    /** The C++ host model of a built-in Gaussian form (svgd_model_create;
     *  built on first use), for svgd_step_host_model / svgd_set_device_model;
     *  nullptr for any other model. */
    const void *HostModelHandle()
    {
        if (!IsGaussianForm())
            return nullptr;
        if (!handle_)
            Build();
        return handle_.get();
    }

    /** A built-in Gaussian form (MultivariateNormal or a sum of them): the
     *  batched C++ host gradient, the device model of svgd_set_device_model. */
    bool IsGaussianForm() const { return !means_.empty() && !model_fun_ && !lhs_; }

protected:
    void AddGaussian(const Eigen::VectorXd &mean, const Eigen::MatrixXd &cov)
    {
        means_.push_back(mean);
        covs_.push_back(cov);
        handle_.reset();
    }
    void RequireGaussian() const
    {
        if (!IsGaussianForm())
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
    std::vector<Eigen::MatrixXd> model_parameters_; // UpdateModel functions' parameters (Model.hpp:458)
    std::shared_ptr<void> handle_;

private:
    /** A model of either kind: a Gaussian form, a set function, a
     *  composition, or a derived class's own EvaluateModel (Model.hpp:63-66
     *  checks the operands' functions are set; a derived class that
     *  overrides the virtuals counts as set). */
    bool HasFunction() const { return IsGaussianForm() || model_fun_ || lhs_ || IsDerived(); }
    bool IsDerived() const { return typeid(*this) != typeid(Model); }

    void CheckComposable(const Model &obj, const char *verb) const
    {
        if (dimension_ != obj.dimension_)
            throw DimensionMismatchException(std::string("Only models with the same variable dimensions can be ") + verb +
                                             ".");
        if (!HasFunction() || !obj.HasFunction())
            throw UnsetException("One of the model functions is unset; functional composition requires both model "
                                 "functions to be set.");
    }

    Model Composed(const Model &obj, char op) const
    {
        Model out((size_t)dimension_);
        out.op_ = op;
        out.lhs_ = CloneSharedPointer();
        out.rhs_ = obj.CloneSharedPointer();
        // a derived model that does not override CloneSharedPointer is
        // sliced to a base Model here.  That is harmless when the slice keeps
        // the behaviour (functions set with UpdateModel, a Gaussian form, a
        // composition: all copied members); a derived model that only
        // overrides the evaluation virtuals would lose them and fail later,
        // inside SVGD::Run: refuse that one now
        auto lost = [](const std::shared_ptr<Model> &clone, const Model &src) {
            return typeid(*clone) != typeid(src) && !clone->HasFunction();
        };
        if (lost(out.lhs_, *this) || lost(out.rhs_, obj))
            throw std::invalid_argument(SVGDCPP_LOG_PREFIX +
                                        "[Argument Error] A derived model must override CloneSharedPointer "
                                        "(returning a copy of its own type) to be composed.");
        return out;
    }

    double Combine(double a, double b) const
    {
        switch (op_)
        {
        case '+': return a + b;
        case '-': return a - b;
        case '*': return a * b;
        default: return a / b;
        }
    }

    ModelFunction model_fun_;
    ModelGradFunction model_grad_fun_;
    ModelHessFunction model_hess_fun_;
    char op_ = 0;                       // composition: + - * /
    std::shared_ptr<Model> lhs_, rhs_; // composition operands (copies)
};

#endif
