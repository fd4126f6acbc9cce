/**
 * @file SVGD.hpp
 * @brief SVGD driver on the MI355X path (reference: include/SVGDCpp/SVGD.hpp:27-511).
 *
 * Same options struct, constructors, checks, messages and Initialize/Run
 * flow as the reference.  Each Step() (SVGD.hpp:373-400) runs on the GPU
 * through the C ABI (svgdcpp_amd/svgd_capi.h):
 *
 *   svgd_begin_step    median-heuristic scale of X_t (GaussianRBFKernel.hpp:141-188)
 *                      while X_t is copied to the host
 *   host               G = grad log p(X_t) from the Model plugin (Model.hpp:335)
 *   svgd_finish_step   phi_hat (SVGD.hpp:407-454), optimizer increment, clamp (:393-399)
 *
 * A built-in Gaussian model (MultivariateNormal or an operator+ sum of them,
 * exactly those types) under the Median or Constant scale takes the one-call
 * step svgd_step_host_model instead: the X_t copy, the host gradient and the
 * G upload pipelined in row chunks behind the device median on a worker
 * thread -- the path bench.py measures; same result bit for bit.
 *
 * The coordinate matrix stays on the device during Run() and is written back
 * to *CoordinateMatrixPtr at the end (the reference mutates it every step).
 *
 * Extensions in SVGDOptions (defaults keep the reference's behaviour): the
 * HIP device, the compute dtype of the O(N^2) work (SVGD_F64 / SVGD_F32),
 * and a sharded run -- World ranks, this process's Rank and the 128-byte
 * RCCL UniqueId (svgd_get_unique_id on one rank, broadcast by the caller):
 * every rank passes the full coordinate matrix, owns rows [row0, row1) of
 * the step and ends Run() with all of them (svgd_create_dist).
 * Requirements of the device path: the kernel is a GaussianRBFKernel
 * (Median, Hessian or Constant scale) and the optimizer is Adam, AdaGrad or
 * RMSProp.  With the Hessian scale, the kernel's model sums -hess log p(X_t)
 * on the host between the two device calls (GaussianRBFKernel.hpp:189-210).
 * LogIntermediateMatrices re-evaluates K and Kg on the host from the step's
 * scale (debug aid for small N, same text format as SVGD.hpp:345-365).
 *
 * Generic kernels: any other Kernel -- a UpdateKernel closed
 * form, a composition, or a derived class overriding EvaluateKernel /
 * EvaluateKernelGrad (Kernel.hpp:279-297) -- runs the reference's serial /
 * parallel ComputePhi on the HOST (SVGD.hpp:373-454: per particle i,
 * UpdateLocation(x_i), then k(x_j, x_i) and grad k(x_j, x_i) for every j),
 * with the plugin optimizer's own Step and the clamp.  The choice is made
 * once, by kernel type, at construction (UsesDevicePath()); a
 * GaussianRBFKernel never takes the host path, and the host path needs no GPU.
 */
#ifndef SVGDCPP_AMD_SVGD_HPP
#define SVGDCPP_AMD_SVGD_HPP

#include <fstream>
#include <exception>
#include <sstream>
#include <typeinfo>

#include "Core.hpp"
#include "Kernel/GaussianRBFKernel.hpp"
#include "Kernel/Kernel.hpp"
#include "Model/Model.hpp"
#include "Model/MultivariateNormal.hpp"
#include "Optimizer/Optimizer.hpp"

/** SVGD.hpp:27-52 (+ Device, ComputeDtype, World / Rank / UniqueId). */
struct SVGDOptions
{
    size_t Dimension;
    size_t NumIterations;
    std::shared_ptr<Eigen::MatrixXd> CoordinateMatrixPtr = nullptr;
    std::shared_ptr<Kernel> KernelPtr = nullptr;
    std::shared_ptr<Model> ModelPtr = nullptr;
    std::shared_ptr<Optimizer> OptimizerPtr = nullptr;
    Eigen::VectorXd LowerBound = Eigen::VectorXd::Constant(1, -INFINITY);
    Eigen::VectorXd UpperBound = Eigen::VectorXd::Constant(1, INFINITY);
    std::string IntermediateMatricesOutputPath = "log.txt";
    bool Parallel = false;
    bool LogIntermediateMatrices = false;
    int Device = 0;
    /** Extension: significant digits of the logged matrices (0 = the stream
     *  default, 6, as the reference writes them). */
    int IntermediateMatricesPrecision = 0;
    /** Extension: compute dtype of the O(N^2) work, SVGD_F64 (the
     *  reference's precision) or SVGD_F32 (svgd_capi.h). */
    int ComputeDtype = SVGD_F64;
    /** Extension: a sharded run over World processes (one GPU each); this
     *  process is Rank.  UniqueId: the 128 bytes of svgd_get_unique_id from
     *  one rank (empty: World must be 1, or the host shared-memory rehearsal
     *  backend SVGD_HOSTCOMM is set). */
    int World = 1;
    int Rank = 0;
    std::vector<unsigned char> UniqueId;
    SVGDOptions() {}
};

class SVGD
{
public:
    SVGD(const SVGDOptions &o)
        : SVGD(o.Dimension, o.NumIterations, o.CoordinateMatrixPtr, o.KernelPtr, o.ModelPtr, o.OptimizerPtr,
               o.LowerBound, o.UpperBound, o.Parallel, o.LogIntermediateMatrices, o.IntermediateMatricesOutputPath,
               o.Device, o.ComputeDtype, o.World, o.Rank, o.UniqueId)
    {
        log_precision_ = o.IntermediateMatricesPrecision;
    }

    SVGD(const size_t &dim, const size_t &iter, const std::shared_ptr<Eigen::MatrixXd> &coord_mat_ptr,
         const std::shared_ptr<Kernel> &kernel_ptr, const std::shared_ptr<Model> &model_ptr,
         const std::shared_ptr<Optimizer> &optimizer_ptr, const bool &parallel = false)
        : SVGD(dim, iter, coord_mat_ptr, kernel_ptr, model_ptr, optimizer_ptr, Eigen::VectorXd::Constant(1, -INFINITY),
               Eigen::VectorXd::Constant(1, INFINITY), parallel)
    {
    }

    SVGD(const size_t &dim, const size_t &iter, const std::shared_ptr<Eigen::MatrixXd> &coord_mat_ptr,
         const std::shared_ptr<Kernel> &kernel_ptr, const std::shared_ptr<Model> &model_ptr,
         const std::shared_ptr<Optimizer> &optimizer_ptr, const Eigen::VectorXd &bound_lower,
         const Eigen::VectorXd &bound_upper, const bool &parallel = false, const bool &log_intermediate_matrices = false,
         const std::string &intermediate_matrices_output_path = "log.txt", int device = 0,
         int compute_dtype = SVGD_F64, int world = 1, int rank = 0,
         const std::vector<unsigned char> &unique_id = {})
        : dimension_((int)coord_mat_ptr->rows()), num_iterations_(iter), parallel_(parallel),
          log_intermediate_matrices_(log_intermediate_matrices),
          intermediate_matrices_output_path_(intermediate_matrices_output_path)
    {
        if ((size_t)dimension_ != dim) // SVGD.hpp:170-173
            throw DimensionMismatchException("Specified dimension does not match the particle coordinate matrix.");
        coord_matrix_ptr_ = coord_mat_ptr;
        num_particles_ = coord_mat_ptr->cols();

        // SVGD.hpp:184-216: bounds enabled unless both are the default 1-row +-inf
        if (bound_lower.rows() == 1 && bound_lower(0) == -INFINITY && bound_upper.rows() == 1 &&
            bound_upper(0) == INFINITY)
        {
            check_bounds_ = false;
        }
        else
        {
            if (bound_lower.rows() != dimension_ && bound_lower.rows() != 1)
                throw DimensionMismatchException("The provided lower bounds have incorrect dimensions.");
            std::cout << SVGDCPP_LOG_PREFIX + "Bound checking enabled, lower bound set to " << bound_lower.transpose()
                      << "." << std::endl;
            if (bound_upper.rows() != dimension_ && bound_upper.rows() != 1)
                throw DimensionMismatchException("The provided upper bounds have incorrect dimensions.");
            std::cout << SVGDCPP_LOG_PREFIX + "Bound checking enabled, upper bound set to " << bound_upper.transpose()
                      << "." << std::endl;
            check_bounds_ = true;
            lower_.assign((size_t)dimension_, 0.0);
            upper_.assign((size_t)dimension_, 0.0);
            for (int k = 0; k < dimension_; ++k)
            {
                lower_[(size_t)k] = bound_lower(bound_lower.rows() == 1 ? 0 : k);
                upper_[(size_t)k] = bound_upper(bound_upper.rows() == 1 ? 0 : k);
            }
        }

        kernel_ptr_ = kernel_ptr;
        model_ptr_ = model_ptr;
        optimizer_ptr_ = optimizer_ptr;
        if (kernel_ptr_ == nullptr) // SVGD.hpp:223-236
            throw std::invalid_argument(SVGDCPP_LOG_PREFIX + "[Argument Error] Invalid Kernel object pointer.");
        if (model_ptr_ == nullptr)
            throw std::invalid_argument(SVGDCPP_LOG_PREFIX + "[Argument Error] Invalid Model object pointer.");
        if (optimizer_ptr_ == nullptr)
            throw std::invalid_argument(SVGDCPP_LOG_PREFIX + "[Argument Error] Invalid Optimizer object pointer.");
        rbf_ptr_ = std::dynamic_pointer_cast<GaussianRBFKernel>(kernel_ptr_);
        if (!rbf_ptr_)
        {
            // generic kernel: the reference's per-pair ComputePhi on the host,
            // the whole problem in this process -- the sharding options
            // (World, Rank, UniqueId) would be silently ignored: refuse them
            if (world > 1 || !unique_id.empty())
                throw std::invalid_argument(SVGDCPP_LOG_PREFIX +
                                            "[Argument Error] World, Rank and UniqueId apply to the GaussianRBFKernel "
                                            "device path only; a generic kernel runs on one host process.");
            std::cout << SVGDCPP_LOG_PREFIX + "Kernel is not a GaussianRBFKernel: phi_hat runs on the host "
                                              "(generic kernel path)."
                      << std::endl;
            return;
        }
        if (optimizer_ptr_->Kind() < 0)
            throw std::invalid_argument(SVGDCPP_LOG_PREFIX +
                                        "[Argument Error] The device path requires Adam, AdaGrad or RMSProp.");
        if (!unique_id.empty() && unique_id.size() != 128)
            throw std::invalid_argument(SVGDCPP_LOG_PREFIX + "[Argument Error] The RCCL unique id has 128 bytes.");
        if (world > 1 && log_intermediate_matrices_)
            throw std::invalid_argument(SVGDCPP_LOG_PREFIX +
                                        "[Argument Error] Intermediate matrices are logged by single-GPU runs only.");

        svgd_ctx *c = nullptr;
        const int rc = world > 1 || !unique_id.empty()
                           ? svgd_create_dist(&c, dimension_, (int64_t)num_particles_, compute_dtype, device, world,
                                              rank, unique_id.empty() ? nullptr : unique_id.data())
                           : svgd_create(&c, dimension_, (int64_t)num_particles_, compute_dtype, device);
        ctx_.reset(c, [](svgd_ctx *p) { svgd_destroy(p); });
        Check(rc);
        Check(svgd_shard(c, &row0_, &row1_));
    }

    SVGD(const SVGD &) = delete;
    ~SVGD() {}

    /** SVGD.hpp:268-296 */
    void Initialize()
    {
        model_ptr_->Initialize();
        kernel_ptr_->Initialize();
        optimizer_ptr_->Initialize();
        if (UsesDevicePath())
            ConfigureDevice();
        if (log_intermediate_matrices_)
        {
            intermediate_matrices_sstream_vector_.clear();
            intermediate_matrices_sstream_vector_.resize(num_iterations_);
        }
        initialized_ = true;
    }

    /** SVGD.hpp:304-320 */
    void UpdateKernelParameters(const std::vector<Eigen::MatrixXd> &params)
    {
        kernel_ptr_->UpdateParameters(params);
        kernel_ptr_->Initialize();
        if (UsesDevicePath())
            ConfigureScale();
    }

    /** SVGD.hpp:328-332 */
    void UpdateModelParameters(const std::vector<Eigen::MatrixXd> &params)
    {
        model_ptr_->UpdateParameters(params);
        model_ptr_->Initialize();
    }

    /** SVGD.hpp:338-366 */
    void Run()
    {
        if (!initialized_)
            throw UnsetException("SVGD::Initialize must be called before Run.");
        if (!UsesDevicePath())
        {
            for (size_t iter = 0; iter < num_iterations_; ++iter)
                HostStep(iter);
            if (log_intermediate_matrices_)
                WriteIntermediateMatricesToFile();
            return;
        }
        svgd_ctx *c = ctx_.get();
        Check(svgd_set_particles(c, coord_matrix_ptr_->data()));
        double *hx = nullptr, *hg = nullptr;
        Check(svgd_host_buffers(c, &hx, &hg));
        for (size_t iter = 0; iter < num_iterations_; ++iter)
        {
            Step(hx, hg);
            if (log_intermediate_matrices_)
                LogStep(iter, hx, hg);
        }
        Check(svgd_get_particles(c, coord_matrix_ptr_->data()));
        if (rbf_ptr_->GetScaleMethod() != GaussianRBFKernel::ScaleMethod::Constant && num_iterations_ > 0)
            rbf_ptr_->UpdateParameters({LastScaleMatrix()});
        if (log_intermediate_matrices_)
            WriteIntermediateMatricesToFile();
    }

    /** The context (for callers that need the C ABI directly); null on the
     *  generic-kernel host path. */
    svgd_ctx *Context() const { return ctx_.get(); }

    /** True for a GaussianRBFKernel (the HIP path), false for the generic
     *  host path of any other kernel. */
    bool UsesDevicePath() const { return rbf_ptr_ != nullptr; }

    /** True when Step() takes the one-call pipelined step (svgd_step_host_model):
     *  a built-in Gaussian model of exactly the Model / MultivariateNormal
     *  type (a subclass may override the gradient or Step(): it keeps the
     *  split calls), the Median or Constant scale, no matrix logging. */
    bool UsesPipelinedStep() const
    {
        if (!UsesDevicePath() || log_intermediate_matrices_ || !model_ptr_->IsGaussianForm())
            return false;
        const Model &m = *model_ptr_;
        if (typeid(m) != typeid(Model) && typeid(m) != typeid(MultivariateNormal))
            return false;
        return rbf_ptr_->GetScaleMethod() != GaussianRBFKernel::ScaleMethod::Hessian;
    }

    /** Rows [row0, row1) of the particles this rank steps (all of them on one GPU). */
    int64_t ShardBegin() const { return row0_; }
    int64_t ShardEnd() const { return row1_; }

protected:
    /** SVGD.hpp:373-400 on the device; the model gradient stays on the host
     *  (this rank's rows).  A built-in Gaussian model takes the pipelined
     *  one-call step (UsesPipelinedStep); any other model the split calls
     *  with its LogModelGradBatch between them. */
    void Step(double *hx, double *hg)
    {
        svgd_ctx *c = ctx_.get();
        model_ptr_->Step();
        if (UsesPipelinedStep())
        {
            Check(svgd_step_host_model(c, model_ptr_->HostModelHandle()));
            return;
        }
        const int64_t rows = row1_ - row0_;
        Check(svgd_begin_step(c, hx));
        if (rbf_ptr_->GetScaleMethod() == GaussianRBFKernel::ScaleMethod::Hessian)
        {
            std::vector<double> H((size_t)dimension_ * dimension_);
            rbf_ptr_->GetTargetModel()->NegHessSumBatch(hx, rows, H.data());
            Check(svgd_set_step_hessian_sum(c, H.data()));
        }
        model_ptr_->LogModelGradBatch(hx, rows, hg);
        Check(svgd_finish_step(c, hg));
    }

    /** The reference's SVGD::Step with ComputePhi (SVGD.hpp:373-454) for a
     *  generic kernel, on the host: K(j, i) = k(x_j, x_i) and
     *  Kg(j d .. j d + d - 1, i) = grad_{x_j} k(x_j, x_i) with the kernel's
     *  location at x_i, phi_i = (1/N) sum_j (K(j, i) G_j + Kg_j), then
     *  X += optimizer.Step(phi) and the clamp.  Parallel mode gives every
     *  OpenMP thread its own kernel clone (the reference clones per particle,
     *  SVGD.hpp:245-248). */
    void HostStep(size_t iter)
    {
        Eigen::MatrixXd &X = *coord_matrix_ptr_;
        const long n = (long)num_particles_, d = dimension_;
        model_ptr_->Step();
        kernel_ptr_->Step();
        Eigen::MatrixXd G(d, n), phi(d, n);
        model_ptr_->LogModelGradBatch(X.data(), n, G.data());
        const bool log = log_intermediate_matrices_;
        Eigen::MatrixXd K, Kg;
        if (log)
        {
            K.resize(n, n);
            Kg.resize(d * n, n);
        }
        const double inv_n = 1.0 / (double)n;
        auto row = [&](Kernel &k, long i) {
            k.UpdateLocation(X.col(i));
            k.Initialize();
            std::vector<double> acc((size_t)d, 0.0);
            for (long j = 0; j < n; ++j)
            {
                const Eigen::VectorXd xj = X.col(j);
                const double kv = k.EvaluateKernel(xj);
                const Eigen::VectorXd kg = k.EvaluateKernelGrad(xj);
                for (long q = 0; q < d; ++q)
                    acc[(size_t)q] += G(q, j) * kv + kg(q);
                if (log)
                {
                    K(j, i) = kv;
                    for (long q = 0; q < d; ++q)
                        Kg(j * d + q, i) = kg(q);
                }
            }
            for (long q = 0; q < d; ++q)
                phi(q, i) = inv_n * acc[(size_t)q];
        };
#ifdef _OPENMP
        if (parallel_)
        {
            // an exception may not leave an OpenMP region (std::terminate):
            // the first one is kept and rethrown after it, as the serial path
            // would throw it
            std::exception_ptr first;
#pragma omp parallel
            {
                try
                {
                    std::unique_ptr<Kernel> k = kernel_ptr_->CloneUniquePointer();
#pragma omp for schedule(static)
                    for (long i = 0; i < n; ++i)
                    {
                        bool skip;
#pragma omp atomic read
                        skip = failed_;
                        if (!skip)
                        {
                            try
                            {
                                row(*k, i);
                            }
                            catch (...)
                            {
#pragma omp critical(svgdcpp_host_step)
                                if (!first)
                                    first = std::current_exception();
#pragma omp atomic write
                                failed_ = true;
                            }
                        }
                    }
                }
                catch (...) // the clone itself
                {
#pragma omp critical(svgdcpp_host_step)
                    if (!first)
                        first = std::current_exception();
#pragma omp atomic write
                    failed_ = true;
                }
            }
            failed_ = false;
            if (first)
                std::rethrow_exception(first);
        }
        else
#endif
        {
            for (long i = 0; i < n; ++i)
                row(*kernel_ptr_, i);
        }
        X += optimizer_ptr_->Step(phi);
        if (check_bounds_)
            for (long i = 0; i < n; ++i)
                for (long q = 0; q < d; ++q)
                    X(q, i) = std::max(std::min(X(q, i), upper_[(size_t)q]), lower_[(size_t)q]);
        if (log)
            LogMatrices(iter, G, K, Kg, X);
    }

    void LogMatrices(size_t iter, const Eigen::MatrixXd &G, const Eigen::MatrixXd &K, const Eigen::MatrixXd &Kg,
                     const Eigen::MatrixXd &X)
    {
        std::stringstream &ss = intermediate_matrices_sstream_vector_[iter];
        if (log_precision_ > 0)
            ss.precision(log_precision_);
        ss << "========== Step " << iter + 1 << " =========="
           << "\nLogModelGrad=\n" << G << "\n\nKernel=\n" << K << "\n\nKernelGrad=\n" << Kg << "\n\nCoordMat=\n" << X
           << "\n\n";
    }

    void ConfigureDevice()
    {
        svgd_ctx *c = ctx_.get();
        double p[4];
        optimizer_ptr_->Params(p);
        Check(svgd_set_optimizer(c, optimizer_ptr_->Kind(), p[0], p[1], p[2], p[3]));
        Check(check_bounds_ ? svgd_set_bounds(c, lower_.data(), upper_.data()) : svgd_set_bounds(c, nullptr, nullptr));
        ConfigureScale();
    }

    void ConfigureScale()
    {
        switch (rbf_ptr_->GetScaleMethod())
        {
        case GaussianRBFKernel::ScaleMethod::Constant:
            if (rbf_ptr_->IsIsotropic())
                Check(svgd_set_scale(ctx_.get(), SVGD_SCALE_FIXED, rbf_ptr_->GetScale()));
            else
            {
                const Eigen::MatrixXd &M = rbf_ptr_->GetScaleMatrix();
                std::vector<double> m((size_t)dimension_ * dimension_);
                for (int r = 0; r < dimension_; ++r)
                    for (int q = 0; q < dimension_; ++q)
                        m[(size_t)r * dimension_ + q] = M(r, q);
                Check(svgd_set_scale_matrix(ctx_.get(), m.data()));
            }
            break;
        case GaussianRBFKernel::ScaleMethod::Hessian:
            Check(svgd_set_scale(ctx_.get(), SVGD_SCALE_HESSIAN, 0.0));
            break;
        default:
            Check(svgd_set_scale(ctx_.get(), SVGD_SCALE_MEDIAN, 0.0));
        }
    }

    /** M of the last step (svgd_get_scale_matrix; row-major -> matrix). */
    Eigen::MatrixXd LastScaleMatrix()
    {
        std::vector<double> m((size_t)dimension_ * dimension_);
        Check(svgd_get_scale_matrix(ctx_.get(), m.data()));
        Eigen::MatrixXd M(dimension_, dimension_);
        for (int r = 0; r < dimension_; ++r)
            for (int q = 0; q < dimension_; ++q)
                M(r, q) = m[(size_t)r * dimension_ + q];
        return M;
    }

    /** SVGD.hpp:345-358 text format; K and Kg re-evaluated on the host. */
    void LogStep(size_t iter, const double *hx, const double *hg)
    {
        const long n = (long)num_particles_, d = dimension_;
        const Eigen::MatrixXd M = LastScaleMatrix();
        Eigen::MatrixXd G(d, n), K(n, n), Kg(d * n, n), X(d, n);
        std::copy(hg, hg + n * d, G.data());
        std::vector<double> diff((size_t)d), Md((size_t)d);
        for (long i = 0; i < n; ++i)
            for (long j = 0; j < n; ++j)
            {
                for (long k = 0; k < d; ++k)
                    diff[(size_t)k] = hx[j * d + k] - hx[i * d + k];
                double u = 0.0;
                for (long r = 0; r < d; ++r)
                {
                    double t = 0.0;
                    for (long q = 0; q < d; ++q)
                        t += M(r, q) * diff[(size_t)q];
                    Md[(size_t)r] = t;
                    u += diff[(size_t)r] * t;
                }
                const double kv = std::exp(-u);
                K(j, i) = kv;
                for (long k = 0; k < d; ++k)
                    Kg(j * d + k, i) = -2.0 * Md[(size_t)k] * kv;
            }
        Check(svgd_get_particles(ctx_.get(), X.data()));
        LogMatrices(iter, G, K, Kg, X);
    }

    /** SVGD.hpp:460-476 */
    void WriteIntermediateMatricesToFile()
    {
        std::ofstream output_file(intermediate_matrices_output_path_);
        if (!output_file)
            throw std::runtime_error(SVGDCPP_LOG_PREFIX + "[Runtime Error] Cannot open " +
                                     intermediate_matrices_output_path_ + " for writing.");
        for (const auto &ss : intermediate_matrices_sstream_vector_)
            output_file << ss.str();
    }

    void Check(int rc) const
    {
        if (rc != SVGD_OK)
            svgdcpp::ThrowFromCode(rc, svgd_last_error(ctx_.get()));
    }

    int dimension_ = -1;
    size_t num_iterations_;
    size_t num_particles_ = 0;
    const bool parallel_ = false;
    bool failed_ = false; // parallel HostStep: a row threw, the others stop
    bool check_bounds_ = false;
    bool log_intermediate_matrices_ = false;
    bool initialized_ = false;
    int log_precision_ = 0;
    int64_t row0_ = 0, row1_ = 0;
    std::vector<double> lower_, upper_;
    std::shared_ptr<Kernel> kernel_ptr_;
    std::shared_ptr<GaussianRBFKernel> rbf_ptr_;
    std::shared_ptr<Model> model_ptr_;
    std::shared_ptr<Optimizer> optimizer_ptr_;
    std::shared_ptr<Eigen::MatrixXd> coord_matrix_ptr_;
    std::shared_ptr<svgd_ctx> ctx_;
    std::vector<std::stringstream> intermediate_matrices_sstream_vector_;
    std::string intermediate_matrices_output_path_ = "log.txt";
};

#endif
