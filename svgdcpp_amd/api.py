"""Python mirror of the reference's plugin API for the SVGD hot path.

Same class / method names, argument meaning and error behaviour as the
reference C++ headers (khaiyichin/SVGDCpp, include/SVGDCpp/...), so tests and
the bench read like the reference's own examples and tests:

    model  = MultivariateNormal(mean, cov)            Model/MultivariateNormal.hpp:39-64
    gmm    = mvn1 + mvn2                               Model/Model.hpp:55-92
    kernel = GaussianRBFKernel(x0, ScaleMethod.Median, model)   Kernel/GaussianRBFKernel.hpp:47-88
    opt    = Adam(dim, n, lr, b1, b2)                  Optimizer/Adam.hpp:33-49
    svgd   = SVGD(dim, iters, x0, kernel, model, opt)  SVGD.hpp:118-250
    svgd.Initialize(); svgd.Run()                      SVGD.hpp:268-366

The coordinate matrix is a numpy array of shape (d, n) -- rows = dimension,
columns = particles, like the reference's Eigen::MatrixXd -- and is updated in
place at the end of Run(), as the reference mutates *coord_matrix_ptr_.

Everything on the hot path (median scale, phi_hat, optimizer, clamp) runs in
the HIP library through the C ABI; the model log-gradient stays on the host
(Model.hpp:335).  Built-in models evaluate it in C++ (svgd_model_* in the C
ABI); user models subclass Model and override EvaluateLogModelGrad (or the
batched log_model_grad).
"""
from __future__ import annotations

import ctypes
import enum
import math

import numpy as np

from . import _capi as C

PREFIX = "SVGDCpp: "


class DimensionMismatchException(Exception):
    """Exceptions.hpp:23-36."""

    def __init__(self, message):
        super().__init__(PREFIX + "[Dimension Error] " + message)


class UnsetException(Exception):
    """Exceptions.hpp:43-56."""

    def __init__(self, message):
        super().__init__(PREFIX + "[Unset Error] " + message)


class DeviceError(RuntimeError):
    pass


def _raise(ctx, rc):
    if rc == C.SVGD_OK:
        return
    msg = C.lib().svgd_last_error(ctx).decode() if ctx else PREFIX + "error"
    if rc == C.SVGD_ERR_DIM:
        e = DimensionMismatchException("")
        e.args = (msg,)
        raise e
    if rc == C.SVGD_ERR_UNSET:
        e = UnsetException("")
        e.args = (msg,)
        raise e
    if rc == C.SVGD_ERR_ARG:
        raise ValueError(msg)
    raise DeviceError(msg)


# ------------------------------------------------------------------ models --

class Model:
    """Model base (Model.hpp:20-494): host-side target density.

    Subclasses override EvaluateLogModelGrad(x) (one particle, d-vector) or the
    batched log_model_grad(X) (X: (n, d) particle rows -> (n, d))."""

    def __init__(self, dim: int = -1):
        self.dimension_ = int(dim)

    def Initialize(self):
        if self.dimension_ <= 0:  # Model.hpp:271-274
            raise UnsetException(f"Model dimension ({self.dimension_}) is improperly or not set.")

    def Step(self):  # Model.hpp:413
        pass

    def EvaluateLogModelGrad(self, x):
        raise UnsetException("Model function is unset.")

    def log_model_grad(self, X):
        X = np.asarray(X, dtype=np.float64)
        return np.stack([np.asarray(self.EvaluateLogModelGrad(x), dtype=np.float64) for x in X])

    def EvaluateLogModelHessian(self, x):  # Model.hpp:366-370
        raise UnsetException("Model function is unset.")

    def neg_hess_sum(self, X):
        """sum_i -hess log p(x_i): the sum inside the Hessian kernel scale."""
        X = np.asarray(X, dtype=np.float64)
        H = np.zeros((self.dimension_, self.dimension_))
        for x in X:
            H -= np.asarray(self.EvaluateLogModelHessian(x), dtype=np.float64)
        return H

    def __add__(self, other):  # Model.hpp:55-92
        if not isinstance(other, Model) or self.dimension_ != other.dimension_:
            raise DimensionMismatchException("Only models with the same variable dimensions can be added.")
        comps = _gaussian_components(self), _gaussian_components(other)
        if comps[0] is None or comps[1] is None:
            raise UnsetException("One of the model functions is unset; functional composition "
                                 "requires both model functions to be set.")
        return GaussianSum(comps[0][0] + comps[1][0], comps[0][1] + comps[1][1])


class GaussianSum(Model):
    """Sum of unnormalised Gaussians exp(-½ (x-μ)ᵀΣ⁻¹(x-μ)); one component is
    MultivariateNormal, several the reference's operator+ composition.  The
    log-gradient is evaluated by the C++ host model (svgd_model_logp_grad)."""

    def __init__(self, means, covariances):
        means = [np.asarray(m, dtype=np.float64).reshape(-1) for m in means]
        covs = [np.asarray(c, dtype=np.float64) for c in covariances]
        d = means[0].shape[0]
        for m, c in zip(means, covs):
            if m.shape[0] != d or c.shape != (d, d):
                raise DimensionMismatchException("Dimensions of parameter vectors/matrices do not match.")
        super().__init__(d)
        self.means_, self.covs_ = means, covs
        self._handle = None
        self._build()

    def _build(self):
        self._free()
        mus = np.ascontiguousarray(np.stack(self.means_))
        covs = np.ascontiguousarray(np.stack(self.covs_))
        h = ctypes.c_void_p()
        rc = C.lib().svgd_model_create(ctypes.byref(h), self.dimension_, len(self.means_),
                                       C.dptr(mus), C.dptr(covs))
        if rc != C.SVGD_OK:
            raise ValueError(PREFIX + "[Argument Error] Singular covariance matrix.")
        self._handle = h

    def _free(self):
        if getattr(self, "_handle", None):
            C.lib().svgd_model_destroy(self._handle)
            self._handle = None

    def __del__(self):
        try:
            self._free()
        except Exception:
            pass

    def log_model_grad(self, X, out=None):
        X = np.ascontiguousarray(X, dtype=np.float64)
        n = X.shape[0]
        G = out if out is not None else np.empty_like(X)
        C.lib().svgd_model_logp_grad(self._handle, C.dptr(X), n, C.dptr(G))
        return G

    def log_model_grad_ptr(self, x_ptr, n, g_ptr):
        C.lib().svgd_model_logp_grad(self._handle, x_ptr, n, g_ptr)

    def EvaluateLogModelGrad(self, x):
        return self.log_model_grad(np.asarray(x, dtype=np.float64).reshape(1, -1))[0]

    def neg_hess_sum(self, X):
        X = np.ascontiguousarray(X, dtype=np.float64)
        H = np.empty((self.dimension_, self.dimension_))
        C.lib().svgd_model_neg_hess_sum(self._handle, C.dptr(X), X.shape[0], C.dptr(H))
        return H

    def neg_hess_sum_ptr(self, x_ptr, n):
        H = np.empty((self.dimension_, self.dimension_))
        C.lib().svgd_model_neg_hess_sum(self._handle, x_ptr, n, C.dptr(H))
        return H

    def EvaluateLogModelHessian(self, x):
        return -self.neg_hess_sum(np.asarray(x, dtype=np.float64).reshape(1, -1))

    def EvaluateLogModel(self, x):
        x = np.asarray(x, dtype=np.float64).reshape(-1)
        q = [0.5 * (x - m) @ np.linalg.solve(c, x - m) for m, c in zip(self.means_, self.covs_)]
        qm = min(q)
        return -qm + math.log(sum(math.exp(-(v - qm)) for v in q))

    def EvaluateModel(self, x):
        return math.exp(self.EvaluateLogModel(x))


class MultivariateNormal(GaussianSum):
    """MultivariateNormal.hpp:23-189 (unnormalised density)."""

    def __init__(self, mean, covariance):
        mean = np.asarray(mean, dtype=np.float64).reshape(-1)
        cov = np.asarray(covariance, dtype=np.float64)
        if cov.ndim != 2 or cov.shape[0] != mean.shape[0] or cov.shape[1] != mean.shape[0]:
            raise DimensionMismatchException("Dimensions of parameter vectors/matrices do not match.")
        super().__init__([mean], [cov])

    def UpdateParameters(self, params):  # MultivariateNormal.hpp:94-115
        mean = np.asarray(params[0], dtype=np.float64).reshape(-1)
        cov = np.asarray(params[1], dtype=np.float64)
        if cov.shape[0] != mean.shape[0] or cov.shape[1] != mean.shape[0]:
            raise DimensionMismatchException(
                "Dimensions of parameter vectors/matrices do not match each other (# of rows must be equal).")
        if mean.shape[0] != self.dimension_:
            raise DimensionMismatchException("Dimensions of parameter vectors/matrices do not match original dimension.")
        self.means_, self.covs_ = [mean], [cov]
        self._build()

    def GetNormalizationConstant(self):  # MultivariateNormal.hpp:182-186
        return 1.0 / ((2.0 * math.pi) ** (self.dimension_ / 2.0) * math.sqrt(np.linalg.det(self.covs_[0])))


def _gaussian_components(m):
    if isinstance(m, GaussianSum):
        return list(m.means_), list(m.covs_)
    return None


# ----------------------------------------------------------------- kernels --

class Kernel:
    """Kernel base (Kernel.hpp:19-420).  Only the Gaussian RBF kernel has a
    device implementation; a plain Kernel cannot drive SVGD here."""

    def __init__(self, dim: int = -1):
        self.dimension_ = int(dim)

    def Initialize(self):
        pass

    def Step(self):
        pass


class GaussianRBFKernel(Kernel):
    """GaussianRBFKernel.hpp:22-270: k(x, x') = exp(-(x-x')ᵀ M (x-x')).

    ScaleMethod.Median recomputes M = a I, a = ln(N)/med², every step on the
    device; ScaleMethod.Hessian recomputes M = Σ_i -∇²log p(x_i) / (2dN)
    every step (:189-210; the model supplies the Hessian on the host);
    ScaleMethod.Constant (extension; the reference's "TODO: constant scale")
    keeps a fixed M set by UpdateParameters([M]) -- isotropic a I or any
    symmetric positive-definite matrix."""

    class ScaleMethod(enum.IntEnum):
        Median = 0
        Hessian = 1
        Constant = 2

    def __init__(self, coord_matrix, method=None, model=None, scale: float = 1.0):
        method = GaussianRBFKernel.ScaleMethod.Median if method is None else method
        super().__init__(np.asarray(coord_matrix).shape[0])
        if method == GaussianRBFKernel.ScaleMethod.Hessian and model is None:
            raise UnsetException("Hessian-based scale requires a model.")
        if method not in tuple(GaussianRBFKernel.ScaleMethod):
            raise ValueError(PREFIX + "[Argument error] Invalid scale method Enum provided.")
        self.scale_method_ = method
        self.coord_matrix_ = coord_matrix
        self.target_model_ = model
        self.scale_ = float(scale)
        self.scale_matrix_ = None  # full M for ScaleMethod.Constant

    def UpdateParameters(self, params):
        M = np.asarray(params[0], dtype=np.float64)
        if M.ndim == 0:
            self.scale_, self.scale_matrix_ = float(M), None
            return
        if M.shape != (self.dimension_, self.dimension_):
            raise DimensionMismatchException("Kernel scale matrix has incorrect dimensions.")
        a = float(M[0, 0])
        if np.array_equal(M, a * np.eye(M.shape[0])):
            self.scale_, self.scale_matrix_ = a, None
        else:
            self.scale_matrix_ = M.copy()


# -------------------------------------------------------------- optimizers --

class Optimizer:
    """Optimizer.hpp:19-48."""

    kind = -1

    def __init__(self, lr, epsilon=1.0e-8):
        self.learning_rate_ = float(lr)
        self.stabilizer_ = float(epsilon)

    def Initialize(self):
        pass


class Adam(Optimizer):
    """Adam.hpp:22-112."""

    kind = C.SVGD_OPT_ADAM

    def __init__(self, dimension, num_particles, lr, beta1, beta2, epsilon=1.0e-8):
        super().__init__(lr, epsilon)
        if beta1 >= 1.0 or beta1 < 0.0 or beta2 >= 1.0 or beta2 < 0.0:
            raise ValueError(PREFIX + "[Argument Error] Invalid value for decay parameter beta.")
        self.dimension_, self.num_particles_ = dimension, num_particles
        self.decay_rate_1_, self.decay_rate_2_ = float(beta1), float(beta2)

    def params(self):
        return (self.learning_rate_, self.decay_rate_1_, self.decay_rate_2_, self.stabilizer_)


class AdaGrad(Optimizer):
    """AdaGrad.hpp:22-76."""

    kind = C.SVGD_OPT_ADAGRAD

    def __init__(self, dimension, num_particles, lr, epsilon=1.0e-8):
        super().__init__(lr, epsilon)
        self.dimension_, self.num_particles_ = dimension, num_particles

    def params(self):
        return (self.learning_rate_, 0.0, 0.0, self.stabilizer_)


class RMSProp(Optimizer):
    """RMSProp.hpp:22-85."""

    kind = C.SVGD_OPT_RMSPROP

    def __init__(self, dimension, num_particles, lr, beta, epsilon=1.0e-8):
        super().__init__(lr, epsilon)
        if beta > 1.0 or beta < 0.0:
            raise ValueError(PREFIX + "[Argument Error] Invalid value for decay parameter beta.")
        self.dimension_, self.num_particles_ = dimension, num_particles
        self.decay_rate_ = float(beta)

    def params(self):
        return (self.learning_rate_, self.decay_rate_, 0.0, self.stabilizer_)


# --------------------------------------------------------------- the driver --

class SVGDOptions:
    """SVGD.hpp:27-52 (+ device selection)."""

    def __init__(self):
        self.Dimension = 0
        self.NumIterations = 0
        self.CoordinateMatrixPtr = None
        self.KernelPtr = None
        self.ModelPtr = None
        self.OptimizerPtr = None
        self.LowerBound = np.array([-np.inf])
        self.UpperBound = np.array([np.inf])
        self.IntermediateMatricesOutputPath = "log.txt"
        self.Parallel = False
        self.LogIntermediateMatrices = False
        self.Device = 0


class Context:
    """Owns one svgd_ctx (one GPU).  Thin RAII wrapper used by SVGD and the bench."""

    def __init__(self, dim, n, device=0, world=1, rank=0, unique_id=None, dtype=None):
        self.lib = C.lib()
        h = ctypes.c_void_p()
        dt = C.SVGD_F64 if dtype is None else int(dtype)
        if world == 1:
            rc = self.lib.svgd_create(ctypes.byref(h), int(dim), int(n), dt, int(device))
        else:
            rc = self.lib.svgd_create_dist(ctypes.byref(h), int(dim), int(n), dt,
                                           int(device), int(world), int(rank), unique_id)
        self.h = h
        if rc != C.SVGD_OK:
            try:
                _raise(h, rc)
            finally:
                self.lib.svgd_destroy(h)
                self.h = None
        r0, r1 = ctypes.c_int64(), ctypes.c_int64()
        self.lib.svgd_shard(self.h, ctypes.byref(r0), ctypes.byref(r1))
        self.row0, self.row1 = r0.value, r1.value
        self.dim, self.n = int(dim), int(n)
        xp, gp = C._D(), C._D()
        self.lib.svgd_host_buffers(self.h, ctypes.byref(xp), ctypes.byref(gp))
        self.x_host_ptr, self.g_host_ptr = xp, gp
        nr = max(1, self.row1 - self.row0)
        self.x_host = np.ctypeslib.as_array(xp, shape=(nr, self.dim))
        self.g_host = np.ctypeslib.as_array(gp, shape=(nr, self.dim))

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        rc = C.lib().svgd_get_unique_id(buf)
        if rc != C.SVGD_OK:
            raise DeviceError(PREFIX + "[RCCL Error] ncclGetUniqueId failed")
        return buf.raw

    def check(self, rc):
        _raise(self.h, rc)

    def close(self):
        if self.h:
            self.lib.svgd_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # thin method wrappers ------------------------------------------------
    def set_particles(self, X_rows):
        X = np.ascontiguousarray(X_rows, dtype=np.float64)
        self.check(self.lib.svgd_set_particles(self.h, C.dptr(X)))

    def get_particles(self):
        X = np.empty((self.n, self.dim))
        self.check(self.lib.svgd_get_particles(self.h, C.dptr(X)))
        return X

    def set_optimizer(self, kind, lr, b1=0.0, b2=0.0, eps=1e-8):
        self.check(self.lib.svgd_set_optimizer(self.h, kind, lr, b1, b2, eps))

    def set_bounds(self, lower, upper):
        if lower is None:
            self.check(self.lib.svgd_set_bounds(self.h, None, None))
            return
        lo = np.ascontiguousarray(lower, dtype=np.float64)
        up = np.ascontiguousarray(upper, dtype=np.float64)
        self.check(self.lib.svgd_set_bounds(self.h, C.dptr(lo), C.dptr(up)))

    def set_scale(self, method, a=1.0):
        self.check(self.lib.svgd_set_scale(self.h, method, a))

    def median_scale(self):
        a, m = ctypes.c_double(), ctypes.c_double()
        self.check(self.lib.svgd_median_scale(self.h, ctypes.byref(a), ctypes.byref(m)))
        return a.value, m.value

    def phi(self, G_shard, a):
        G = np.ascontiguousarray(G_shard, dtype=np.float64)
        out = np.empty((self.row1 - self.row0, self.dim))
        self.check(self.lib.svgd_phi(self.h, C.dptr(G), float(a), C.dptr(out)))
        return out

    def last_scale(self):
        a, m, p = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        self.check(self.lib.svgd_last_scale(self.h, ctypes.byref(a), ctypes.byref(m), ctypes.byref(p)))
        return a.value, m.value, p.value

    def step_with_model(self, model, hessian=False):
        """One SVGD::Step with host gradients from `model` (overlapped with the
        device median via begin/finish).  hessian=True: the Hessian kernel
        scale, with this shard's sum of -hess log p supplied from `model`."""
        self.check(self.lib.svgd_begin_step(self.h, self.x_host_ptr))
        nr = self.row1 - self.row0
        if hessian:
            H = (model.neg_hess_sum_ptr(self.x_host_ptr, nr) if isinstance(model, GaussianSum)
                 else model.neg_hess_sum(self.x_host[:nr]))
            self.set_step_hessian_sum(H)
        if isinstance(model, GaussianSum):
            model.log_model_grad_ptr(self.x_host_ptr, nr, self.g_host_ptr)
        elif nr > 0:
            self.g_host[:nr] = model.log_model_grad(self.x_host[:nr])
        self.check(self.lib.svgd_finish_step(self.h, self.g_host_ptr))

    def set_scale_matrix(self, M):
        M = np.ascontiguousarray(M, dtype=np.float64)
        self.check(self.lib.svgd_set_scale_matrix(self.h, C.dptr(M)))

    def set_step_hessian_sum(self, H):
        H = np.ascontiguousarray(H, dtype=np.float64)
        self.check(self.lib.svgd_set_step_hessian_sum(self.h, C.dptr(H)))

    def get_scale_matrix(self):
        M = np.empty((self.dim, self.dim))
        self.check(self.lib.svgd_get_scale_matrix(self.h, C.dptr(M)))
        return M

    def set_device_model(self, model):
        """Mirror a GaussianSum on the device; then
        step_device() runs the whole step, grad log p included, in HBM."""
        if model is not None and not isinstance(model, GaussianSum):
            raise TypeError("only the built-in Gaussian-sum models have a device form")
        self.check(self.lib.svgd_set_device_model(self.h, model._handle if model is not None else None))
        self._device_model = model  # keep the host handle alive

    def device_logp_grad(self):
        out = np.empty((self.row1 - self.row0, self.dim), dtype=np.float64)
        self.check(self.lib.svgd_device_logp_grad(self.h, C.dptr(out)))
        return out

    def step_device(self):
        self.check(self.lib.svgd_step(self.h, None))

    def sync(self):
        self.check(self.lib.svgd_sync(self.h))


class SVGD:
    """SVGD.hpp:84-511 on the MI355X path.

    Parallel=True is accepted for API compatibility; the device path is
    always parallel.  LogIntermediateMatrices is not supported on the device
    path (it needs the N x N matrices the fused kernel never materialises)."""

    def __init__(self, *args, **kw):
        if len(args) == 1 and isinstance(args[0], SVGDOptions):
            o = args[0]
            args = (o.Dimension, o.NumIterations, o.CoordinateMatrixPtr, o.KernelPtr, o.ModelPtr,
                    o.OptimizerPtr, o.LowerBound, o.UpperBound, o.Parallel,
                    o.LogIntermediateMatrices, o.IntermediateMatricesOutputPath)
            kw.setdefault("device", o.Device)
        dim, iters, coord, kernel, model, opt = args[:6]
        rest = list(args[6:])
        if rest and isinstance(rest[0], (bool, np.bool_)) and len(rest) == 1:
            lower, upper, parallel = np.array([-np.inf]), np.array([np.inf]), rest[0]
            log = False
        else:
            lower = rest[0] if len(rest) > 0 else np.array([-np.inf])
            upper = rest[1] if len(rest) > 1 else np.array([np.inf])
            parallel = rest[2] if len(rest) > 2 else False
            log = rest[3] if len(rest) > 3 else False
        coord = np.asarray(coord)
        self.dimension_ = coord.shape[0]
        if self.dimension_ != dim:  # SVGD.hpp:170-173
            raise DimensionMismatchException("Specified dimension does not match the particle coordinate matrix.")
        self.num_iterations_ = int(iters)
        self.coord_matrix_ = coord
        lower = np.atleast_1d(np.asarray(lower, dtype=np.float64))
        upper = np.atleast_1d(np.asarray(upper, dtype=np.float64))
        if lower.shape == (1,) and upper.shape == (1,) and lower[0] == -np.inf and upper[0] == np.inf:
            self.bounds_ = None  # SVGD.hpp:184-190
        else:
            if lower.shape[0] not in (self.dimension_, 1):
                raise DimensionMismatchException("The provided lower bounds have incorrect dimensions.")
            if upper.shape[0] not in (self.dimension_, 1):
                raise DimensionMismatchException("The provided upper bounds have incorrect dimensions.")
            self.bounds_ = (np.broadcast_to(lower, (self.dimension_,)).copy(),
                            np.broadcast_to(upper, (self.dimension_,)).copy())
        if kernel is None:
            raise ValueError(PREFIX + "[Argument Error] Invalid Kernel object pointer.")
        if model is None:
            raise ValueError(PREFIX + "[Argument Error] Invalid Model object pointer.")
        if opt is None:
            raise ValueError(PREFIX + "[Argument Error] Invalid Optimizer object pointer.")
        if not isinstance(kernel, GaussianRBFKernel):
            raise ValueError(PREFIX + "[Argument Error] The device path needs a GaussianRBFKernel.")
        if log:
            raise ValueError(PREFIX + "[Argument Error] LogIntermediateMatrices is not supported "
                             "on the device path.")
        self.kernel_, self.model_, self.optimizer_ = kernel, model, opt
        self.parallel_ = bool(parallel)
        self.ctx = Context(self.dimension_, coord.shape[1], device=kw.get("device", 0))

    def Initialize(self):
        """SVGD.hpp:268-296: model, kernel and optimizer initialisation."""
        self.model_.Initialize()
        self.kernel_.Initialize()
        self.optimizer_.Initialize()
        c = self.ctx
        c.set_optimizer(self.optimizer_.kind, *self.optimizer_.params())
        c.set_bounds(*(self.bounds_ if self.bounds_ is not None else (None, None)))
        k = self.kernel_
        if k.scale_method_ == GaussianRBFKernel.ScaleMethod.Constant:
            if k.scale_matrix_ is not None:
                c.set_scale_matrix(k.scale_matrix_)
            else:
                c.set_scale(C.SVGD_SCALE_FIXED, k.scale_)
        elif k.scale_method_ == GaussianRBFKernel.ScaleMethod.Hessian:
            c.set_scale(C.SVGD_SCALE_HESSIAN, 0.0)
        else:
            c.set_scale(C.SVGD_SCALE_MEDIAN, 0.0)
        self._initialized = True

    def Run(self):
        """SVGD.hpp:338-366; coordinates are read from / written back to the
        caller's (d, n) matrix."""
        if not getattr(self, "_initialized", False):
            raise UnsetException("SVGD::Initialize must be called before Run.")
        c = self.ctx
        c.set_particles(np.ascontiguousarray(self.coord_matrix_.T))
        hess = self.kernel_.scale_method_ == GaussianRBFKernel.ScaleMethod.Hessian
        hmodel = self.kernel_.target_model_ if hess else None
        for _ in range(self.num_iterations_):
            self.model_.Step()
            if hess and hmodel is not self.model_:
                # the kernel's own model supplies the Hessian (GaussianRBFKernel.hpp:202)
                c.check(c.lib.svgd_begin_step(c.h, c.x_host_ptr))
                nr = c.row1 - c.row0
                c.set_step_hessian_sum(hmodel.neg_hess_sum(c.x_host[:nr]))
                if isinstance(self.model_, GaussianSum):
                    self.model_.log_model_grad_ptr(c.x_host_ptr, nr, c.g_host_ptr)
                elif nr > 0:
                    c.g_host[:nr] = self.model_.log_model_grad(c.x_host[:nr])
                c.check(c.lib.svgd_finish_step(c.h, c.g_host_ptr))
            else:
                c.step_with_model(self.model_, hessian=hess)
        X = c.get_particles()
        self.coord_matrix_[...] = X.T

    def UpdateKernelParameters(self, params):  # SVGD.hpp:304-320
        self.kernel_.UpdateParameters(params)
        self.Initialize()

    def UpdateModelParameters(self, params):  # SVGD.hpp:328-332
        self.model_.UpdateParameters(params)
        self.model_.Initialize()
