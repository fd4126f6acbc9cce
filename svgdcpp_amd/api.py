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

import copy
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

    CppAD is not part of this build, so a model is given in closed form (the
    reference's "Method 3", doc/instructions.md:234-301): a subclass overrides
    EvaluateLogModelGrad(x) (one particle, d-vector) or the batched
    log_model_grad(X) ((n, d) rows -> (n, d)), or -- to compose --
    EvaluateModel / EvaluateModelGrad [/ EvaluateModelHessian]; or the
    function is set with its derivatives, UpdateModel(f, grad_f[, hess_f]),
    each taking (x, params) like the reference's ModelFun (:434-443).
    Composition (+ - * /, :55-227) applies the sum, product and quotient rules
    to the operands' closed forms; log p and its derivatives follow from p
    (grad log p = grad p / p, hess log p = hess p / p - grad p grad p^T / p^2,
    the reference's LogModelFun :451-454).  Two Gaussian forms add into a
    Gaussian form (GaussianSum: the batched C++ host gradient)."""

    def __init__(self, dim: int = -1):
        self.dimension_ = int(dim)
        self.model_parameters_ = []
        self._fun = self._grad = self._hess = None
        self._op, self._lhs, self._rhs = None, None, None

    def Initialize(self):
        if self.dimension_ <= 0:  # Model.hpp:271-274
            raise UnsetException(f"Model dimension ({self.dimension_}) is improperly or not set.")

    def Step(self):  # Model.hpp:413
        pass

    # ---- closed forms (Model.hpp:290-370) ----
    def UpdateModel(self, fun, grad, hess=None):  # Model.hpp:421-424, derivatives in closed form
        self._fun, self._grad, self._hess = fun, grad, hess
        self._op, self._lhs, self._rhs = None, None, None

    def UpdateParameters(self, params):  # Model.hpp:377-388
        if self._lhs is not None:  # the operands' parameters, concatenated (:70-74)
            n1 = len(self._lhs.GetParameters())
            if len(params) != n1 + len(self._rhs.GetParameters()):
                raise DimensionMismatchException("Number of parameters does not match the model.")
            # copy on write: copies of this composition share its operands
            # (the reference's composed model keeps its own parameters, :70-81)
            self._lhs, self._rhs = _clone_model(self._lhs), _clone_model(self._rhs)
            self._lhs.UpdateParameters(list(params[:n1]))
            self._rhs.UpdateParameters(list(params[n1:]))
            return
        self.model_parameters_ = [np.asarray(q, dtype=np.float64) for q in params]

    def GetParameters(self):  # Model.hpp:395-406
        if self._lhs is not None:
            return self._lhs.GetParameters() + self._rhs.GetParameters()
        return list(self.model_parameters_)

    def EvaluateModel(self, x):
        x = np.asarray(x, dtype=np.float64).reshape(-1)
        if self._fun is not None:
            return float(self._fun(x, self.model_parameters_))
        if self._lhs is not None:
            a, b = self._lhs.EvaluateModel(x), self._rhs.EvaluateModel(x)
            return {"+": a + b, "-": a - b, "*": a * b}.get(self._op, a / b if self._op == "/" else None)
        raise UnsetException("Model function is unset.")

    def EvaluateLogModel(self, x):
        return math.log(self.EvaluateModel(x))

    def EvaluateModelGrad(self, x):
        x = np.asarray(x, dtype=np.float64).reshape(-1)
        if self._grad is not None:
            return np.asarray(self._grad(x, self.model_parameters_), dtype=np.float64).reshape(-1)
        if self._lhs is not None:
            a, b = self._lhs.EvaluateModel(x), self._rhs.EvaluateModel(x)
            ga, gb = self._lhs.EvaluateModelGrad(x), self._rhs.EvaluateModelGrad(x)
            if self._op == "+":
                return ga + gb
            if self._op == "-":
                return ga - gb
            if self._op == "*":
                return b * ga + a * gb
            return (b * ga - a * gb) / (b * b)
        raise UnsetException("Model function is unset.")

    def EvaluateModelHessian(self, x):
        x = np.asarray(x, dtype=np.float64).reshape(-1)
        if self._hess is not None:
            return np.asarray(self._hess(x, self.model_parameters_), dtype=np.float64)
        if self._lhs is not None:
            a, b = self._lhs.EvaluateModel(x), self._rhs.EvaluateModel(x)
            ga, gb = self._lhs.EvaluateModelGrad(x), self._rhs.EvaluateModelGrad(x)
            Ha, Hb = self._lhs.EvaluateModelHessian(x), self._rhs.EvaluateModelHessian(x)
            cross = np.outer(ga, gb) + np.outer(gb, ga)
            if self._op == "+":
                return Ha + Hb
            if self._op == "-":
                return Ha - Hb
            if self._op == "*":
                return b * Ha + cross + a * Hb
            return Ha / b - cross / (b * b) + (2.0 * a / b ** 3) * np.outer(gb, gb) - (a / (b * b)) * Hb
        raise UnsetException("Model function is unset.")

    def EvaluateLogModelGrad(self, x):
        return self.EvaluateModelGrad(x) / self.EvaluateModel(x)

    def EvaluateLogModelHessian(self, x):  # Model.hpp:366-370
        p, g = self.EvaluateModel(x), self.EvaluateModelGrad(x)
        return self.EvaluateModelHessian(x) / p - np.outer(g, g) / (p * p)

    def log_model_grad(self, X):
        X = np.asarray(X, dtype=np.float64)
        return np.stack([np.asarray(self.EvaluateLogModelGrad(x), dtype=np.float64) for x in X])

    def neg_hess_sum(self, X):
        """sum_i -hess log p(x_i): the sum inside the Hessian kernel scale."""
        X = np.asarray(X, dtype=np.float64)
        H = np.zeros((self.dimension_, self.dimension_))
        for x in X:
            H -= np.asarray(self.EvaluateLogModelHessian(x), dtype=np.float64)
        return H

    # ---- composition (Model.hpp:55-227) ----
    def _has_function(self):
        t = type(self)
        return (self._fun is not None or self._lhs is not None or t.EvaluateModel is not Model.EvaluateModel
                or t.EvaluateLogModelGrad is not Model.EvaluateLogModelGrad)

    def _compose(self, other, op, verb):
        if not isinstance(other, Model) or self.dimension_ != other.dimension_:
            raise DimensionMismatchException(f"Only models with the same variable dimensions can be {verb}.")
        if not self._has_function() or not other._has_function():
            raise UnsetException("One of the model functions is unset; functional composition "
                                 "requires both model functions to be set.")
        out = Model(self.dimension_)
        # copies of the operands: updating the composition's parameters must
        # not change the models it was built from (Model.hpp:70-81)
        out._op, out._lhs, out._rhs = op, _clone_model(self), _clone_model(other)
        return out

    def __add__(self, other):  # Model.hpp:55-92
        comps = _gaussian_components(self), _gaussian_components(other)
        if (comps[0] is not None and comps[1] is not None and self.dimension_ == other.dimension_
                and all(_builtin_grad(m) and _builtin_hess(m) for m in (self, other))):
            return GaussianSum(comps[0][0] + comps[1][0], comps[0][1] + comps[1][1])
        return self._compose(other, "+", "added")

    def __sub__(self, other):  # Model.hpp:100-137
        return self._compose(other, "-", "added")

    def __mul__(self, other):  # Model.hpp:145-182
        return self._compose(other, "*", "multiplied")

    def __truediv__(self, other):  # Model.hpp:190-227
        return self._compose(other, "/", "multiplied")


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

    def EvaluateModelGrad(self, x):  # p grad log p (an operand of a composition)
        return self.EvaluateModel(x) * self.EvaluateLogModelGrad(x)

    def EvaluateModelHessian(self, x):  # p (hess log p + grad log p grad log p^T)
        g = self.EvaluateLogModelGrad(x)
        return self.EvaluateModel(x) * (self.EvaluateLogModelHessian(x) + np.outer(g, g))

    def UpdateParameters(self, params):  # (mean, covariance) per component, in order
        if len(params) != 2 * len(self.means_):
            raise DimensionMismatchException("Number of parameters does not match the model.")
        means = [np.asarray(m, dtype=np.float64).reshape(-1) for m in params[0::2]]
        covs = [np.asarray(c, dtype=np.float64) for c in params[1::2]]
        for m, c in zip(means, covs):
            if m.shape[0] != self.dimension_ or c.shape != (self.dimension_, self.dimension_):
                raise DimensionMismatchException("Dimensions of parameter vectors/matrices do not match original dimension.")
        self.means_, self.covs_ = means, covs
        self._build()

    def GetParameters(self):  # Model.hpp:395-406: mean0, cov0, mean1, cov1, ...
        out = []
        for m, c in zip(self.means_, self.covs_):
            out += [m.copy(), c.copy()]
        return out


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


def _clone_model(model):
    """A copy of a model that shares no mutable state with it: parameter
    lists and Gaussian components copied, a GaussianSum's C++ host model
    rebuilt (its handle is owned by one object), composed operands cloned in
    turn.  Other attributes of a user subclass are copied shallowly, as a C++
    copy constructor copies its members."""
    c = copy.copy(model)
    c.model_parameters_ = [np.array(q, copy=True) for q in model.model_parameters_]
    if isinstance(model, GaussianSum):
        c.means_ = [m.copy() for m in model.means_]
        c.covs_ = [v.copy() for v in model.covs_]
        c._handle = None  # (never free the original's)
        c._build()
    if model._lhs is not None:
        c._lhs, c._rhs = _clone_model(model._lhs), _clone_model(model._rhs)
    return c


def _builtin_grad(model):
    """The model's gradient is the built-in C++ one: a GaussianSum whose
    subclass (if any) overrides neither gradient method -- only then may the
    C handle evaluate it (an override must run as the user wrote it)."""
    t = type(model)
    return (isinstance(model, GaussianSum) and t.log_model_grad is GaussianSum.log_model_grad
            and t.EvaluateLogModelGrad is GaussianSum.EvaluateLogModelGrad)


def _builtin_hess(model):
    t = type(model)
    return (isinstance(model, GaussianSum) and t.neg_hess_sum is GaussianSum.neg_hess_sum
            and t.EvaluateLogModelHessian is GaussianSum.EvaluateLogModelHessian)


def _gaussian_components(m):
    if isinstance(m, GaussianSum):
        return list(m.means_), list(m.covs_)
    return None


# ----------------------------------------------------------------- kernels --

class Kernel:
    """Kernel base (Kernel.hpp:19-420).

    The Gaussian RBF kernel runs fused on the device.  Any other kernel -- a
    closed form set with UpdateKernel(f, grad_f), a composition k1 + k2,
    k1 - k2, k1 * k2, k1 / k2 (Kernel.hpp:55-223, parameters concatenated), or
    a subclass overriding EvaluateKernel / EvaluateKernelGrad (:279-297) --
    drives SVGD's generic host path (SVGD.Run).  f and grad_f take
    (x, params, location) like the reference's KernelFun (:391-399); there is
    no tape engine, so the gradient is given in closed form."""

    def __init__(self, dim: int = -1):
        self.dimension_ = int(dim)
        self.location_ = np.zeros(max(0, self.dimension_))
        self.kernel_parameters_ = []
        self._fun = None
        self._grad = None

    def Initialize(self):
        pass

    def Step(self):
        pass

    def UpdateKernel(self, kernel_fun, kernel_grad_fun):
        self._fun, self._grad = kernel_fun, kernel_grad_fun

    def UpdateParameters(self, params):
        self.kernel_parameters_ = [np.asarray(p, dtype=np.float64) for p in params]

    def GetParameters(self):
        return list(self.kernel_parameters_)

    def UpdateLocation(self, x):
        x = np.asarray(x, dtype=np.float64).reshape(-1)
        if x.shape[0] != self.dimension_:
            raise DimensionMismatchException(
                f"Dimension mismatch between provided location and kernel dimension "
                f"({x.shape[0]} vs. {self.dimension_}).")
        self.location_ = x

    def EvaluateKernel(self, x):
        if self._fun is None:
            raise UnsetException("Kernel function is unset.")
        return float(self._fun(np.asarray(x, dtype=np.float64), self.kernel_parameters_, self.location_))

    def EvaluateKernelGrad(self, x):
        if self._grad is None:
            raise UnsetException("Kernel function is unset.")
        return np.asarray(self._grad(np.asarray(x, dtype=np.float64), self.kernel_parameters_, self.location_),
                          dtype=np.float64)

    def _compose(self, other, f, g):
        if self.dimension_ != other.dimension_:
            raise DimensionMismatchException("Only kernels with the same variable dimensions can be added.")
        if None in (self._fun, self._grad, other._fun, other._grad):
            raise UnsetException("One of the kernel functions is unset; functional composition requires both "
                                 "kernel functions to be set.")
        n1 = len(self.kernel_parameters_)
        f1, g1, f2, g2 = self._fun, self._grad, other._fun, other._grad
        out = Kernel(self.dimension_)
        out.kernel_parameters_ = list(self.kernel_parameters_) + list(other.kernel_parameters_)
        out._fun = lambda x, p, loc: f(f1(x, p[:n1], loc), f2(x, p[n1:], loc))
        out._grad = lambda x, p, loc: g(f1(x, p[:n1], loc), np.asarray(g1(x, p[:n1], loc)),
                                        f2(x, p[n1:], loc), np.asarray(g2(x, p[n1:], loc)))
        return out

    def __add__(self, other):  # Kernel.hpp:55-88
        return self._compose(other, lambda a, b: a + b, lambda a, ga, b, gb: ga + gb)

    def __sub__(self, other):  # Kernel.hpp:96-129
        return self._compose(other, lambda a, b: a - b, lambda a, ga, b, gb: ga - gb)

    def __mul__(self, other):  # Kernel.hpp:137-170 (product rule)
        return self._compose(other, lambda a, b: a * b, lambda a, ga, b, gb: b * ga + a * gb)

    def __truediv__(self, other):  # Kernel.hpp:178-223 (quotient rule)
        return self._compose(other, lambda a, b: a / b, lambda a, ga, b, gb: (b * ga - a * gb) / (b * b))


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
        self.kernel_parameters_ = [self.scale_matrix()]
        # the closed form as the kernel function too (the reference sets its
        # lambda with UpdateKernel, GaussianRBFKernel.hpp:75-87), so rbf + k,
        # rbf * k, ... compose on the generic host path like any set kernel
        self._fun = GaussianRBFKernel._value
        self._grad = GaussianRBFKernel._gradient

    @staticmethod
    def _value(x, params, loc):  # :75-81, M = params[0]
        diff = np.asarray(x, dtype=np.float64) - loc
        return float(np.exp(-diff @ np.asarray(params[0]) @ diff))

    @staticmethod
    def _gradient(x, params, loc):
        diff = np.asarray(x, dtype=np.float64) - loc
        M = np.asarray(params[0])
        return -2.0 * (M @ diff) * np.exp(-diff @ M @ diff)

    def scale_matrix(self):
        """M of k(x, x') = exp(-(x-x')^T M (x-x'))."""
        if self.scale_matrix_ is not None:
            return self.scale_matrix_
        return self.scale_ * np.eye(self.dimension_)

    def EvaluateKernel(self, x):  # GaussianRBFKernel.hpp:75-81
        return self._value(x, [self.scale_matrix()], self.location_)

    def EvaluateKernelGrad(self, x):
        return self._gradient(x, [self.scale_matrix()], self.location_)

    def UpdateParameters(self, params):
        M = np.asarray(params[0], dtype=np.float64)
        if M.ndim == 0:
            self.scale_, self.scale_matrix_ = float(M), None
        elif M.shape != (self.dimension_, self.dimension_):
            raise DimensionMismatchException("Kernel scale matrix has incorrect dimensions.")
        else:
            a = float(M[0, 0])
            if np.array_equal(M, a * np.eye(M.shape[0])):
                self.scale_, self.scale_matrix_ = a, None
            else:
                self.scale_matrix_ = M.copy()
        self.kernel_parameters_ = [self.scale_matrix()]


# -------------------------------------------------------------- optimizers --

class Optimizer:
    """Optimizer.hpp:19-48."""

    kind = -1

    def __init__(self, lr, epsilon=1.0e-8):
        self.learning_rate_ = float(lr)
        self.stabilizer_ = float(epsilon)
        self.counter_ = 0
        self.m_ = self.v_ = None

    def Initialize(self):
        """Optimizer.hpp:35: zero the state (the device path keeps its own copy)."""
        self.counter_ = 0
        self.m_ = self.v_ = None

    def Step(self, grad):
        """Optimizer.hpp:42: the increment for grad (d, n) -- used on the
        generic-kernel host path; the device path runs the same update fused."""
        raise NotImplementedError


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

    def Step(self, g):  # Adam.hpp:75-96
        g = np.asarray(g, dtype=np.float64)
        if self.m_ is None:
            self.m_, self.v_ = np.zeros_like(g), np.zeros_like(g)
        b1, b2 = self.decay_rate_1_, self.decay_rate_2_
        self.m_ = b1 * self.m_ + (1 - b1) * g
        self.v_ = b2 * self.v_ + (1 - b2) * (g * g)
        self.counter_ += 1
        c1, c2 = 1.0 - b1 ** self.counter_, 1.0 - b2 ** self.counter_
        return (self.learning_rate_ * (1.0 / (self.stabilizer_ + np.sqrt(self.v_ / c2)))) * (self.m_ / c1)


class AdaGrad(Optimizer):
    """AdaGrad.hpp:22-76."""

    kind = C.SVGD_OPT_ADAGRAD

    def __init__(self, dimension, num_particles, lr, epsilon=1.0e-8):
        super().__init__(lr, epsilon)
        self.dimension_, self.num_particles_ = dimension, num_particles

    def params(self):
        return (self.learning_rate_, 0.0, 0.0, self.stabilizer_)

    def Step(self, g):  # AdaGrad.hpp:60-65
        g = np.asarray(g, dtype=np.float64)
        if self.v_ is None:
            self.v_ = np.zeros_like(g)
        self.v_ = self.v_ + g * g
        return self.learning_rate_ * g / (self.stabilizer_ + np.sqrt(self.v_))


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

    def Step(self, g):  # RMSProp.hpp:69-74
        g = np.asarray(g, dtype=np.float64)
        if self.v_ is None:
            self.v_ = np.zeros_like(g)
        b = self.decay_rate_
        self.v_ = b * self.v_ + (1 - b) * (g * g)
        return self.learning_rate_ * g / (self.stabilizer_ + np.sqrt(self.v_))


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
        self.IntermediateMatricesPrecision = 0  # extension: digits of the log (0 = 6, the reference's)
        self.Parallel = False
        self.LogIntermediateMatrices = False
        self.Device = 0


class Context:
    """Owns one svgd_ctx (one GPU).  Thin RAII wrapper used by SVGD and the bench."""

    def __init__(self, dim, n, device=0, world=1, rank=0, unique_id=None, dtype=None, sim_world=None):
        """sim_world=P (measurement only): svgd_create_sim -- rank 0's share of
        a P-rank step on one GPU; result calls on it raise."""
        self.lib = C.lib()
        h = ctypes.c_void_p()
        dt = C.SVGD_F64 if dtype is None else int(dtype)
        if sim_world is not None and sim_world > 1:
            if world != 1:
                raise ValueError("sim_world is a one-rank measurement context")
            rc = self.lib.svgd_create_sim(ctypes.byref(h), int(dim), int(n), dt, int(device), int(sim_world))
        elif world == 1 and unique_id is None:
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

    def last_median_keys(self):
        """(sq_lo, sq_hi, rank_lo, rank_hi): the upper-list order statistics
        (squared distances) the last median averaged, and their ranks."""
        a, b = ctypes.c_double(), ctypes.c_double()
        r0, r1 = ctypes.c_int64(), ctypes.c_int64()
        self.check(self.lib.svgd_last_median_keys(self.h, ctypes.byref(a), ctypes.byref(b),
                                                  ctypes.byref(r0), ctypes.byref(r1)))
        return a.value, b.value, r0.value, r1.value

    def set_median_tuning(self, direct_max_pairs=-1, sample_size=-1, candidate_capacity=-1):
        self.check(self.lib.svgd_set_median_tuning(self.h, int(direct_max_pairs), int(sample_size),
                                                   int(candidate_capacity)))

    def step_with_model(self, model, hessian=False, pipelined=True):
        """One SVGD::Step with host gradients from `model` (overlapped with the
        device median via begin/finish).  hessian=True: the Hessian kernel
        scale, with this shard's sum of -hess log p supplied from `model`.
        A built-in GaussianSum runs through svgd_step_host_model (the X_t copy,
        the gradient and the G upload pipelined in row chunks, all in C; the
        host buffers x_host / g_host are then not guaranteed to hold X_t);
        pipelined=False takes the split begin / gradient / finish calls."""
        if pipelined and not hessian and _builtin_grad(model):
            self.check(self.lib.svgd_step_host_model(self.h, model._handle))
            return
        self.check(self.lib.svgd_begin_step(self.h, self.x_host_ptr))
        nr = self.row1 - self.row0
        if hessian:
            H = (model.neg_hess_sum_ptr(self.x_host_ptr, nr) if _builtin_hess(model)
                 else model.neg_hess_sum(self.x_host[:nr]))
            self.set_step_hessian_sum(H)
        if _builtin_grad(model):
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
        if model is not None and not _builtin_grad(model):
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

    def phi_kernel_name(self):
        """The phi kernel (name<template args>) this context launches."""
        buf = ctypes.create_string_buffer(128)
        self.check(self.lib.svgd_phi_kernel_name(self.h, buf, 128))
        return buf.value.decode()

    def diagnostics(self):
        """svgd_get_diagnostics as a dict (accumulated since the last call, then reset)."""
        buf = (ctypes.c_double * C.SVGD_DIAG_LEN)()
        rc = self.lib.svgd_get_diagnostics(self.h, buf, C.SVGD_DIAG_LEN)
        if rc < 0:
            self.check(rc)
        return dict(zip(C.DIAG_NAMES, list(buf)))


class SVGD:
    """SVGD.hpp:84-511 on the MI355X path.

    A GaussianRBFKernel runs every step on the device (UsesDevicePath()).  Any
    other kernel runs the reference's ComputePhi on the host (the generic
    kernel path, SURVEY 8(f) 4: SVGD.hpp:407-454 with the kernel's location
    at each x_i, then the optimizer's own Step and the clamp); the choice is
    made by kernel type at construction.  Parallel=True is accepted for API
    compatibility.  LogIntermediateMatrices writes the reference's text
    format (SVGD.hpp:345-365, 460-476); on the device path K and Kg are
    re-evaluated on the host from the step's scale (small N only)."""

    def __init__(self, *args, **kw):
        if len(args) == 1 and isinstance(args[0], SVGDOptions):
            o = args[0]
            args = (o.Dimension, o.NumIterations, o.CoordinateMatrixPtr, o.KernelPtr, o.ModelPtr,
                    o.OptimizerPtr, o.LowerBound, o.UpperBound, o.Parallel,
                    o.LogIntermediateMatrices, o.IntermediateMatricesOutputPath)
            kw.setdefault("device", o.Device)
            kw.setdefault("log_precision", o.IntermediateMatricesPrecision)
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
        self.kernel_, self.model_, self.optimizer_ = kernel, model, opt
        self.parallel_ = bool(parallel)
        self.log_ = bool(log)
        self.log_path_ = (args[10] if len(args) > 10 else kw.get("log_path", "log.txt"))
        self.log_precision_ = int(kw.get("log_precision", 0))
        self.logs_ = []
        self.ctx = None
        if isinstance(kernel, GaussianRBFKernel):
            self.ctx = Context(self.dimension_, coord.shape[1], device=kw.get("device", 0))
        elif not hasattr(opt, "Step"):
            raise ValueError(PREFIX + "[Argument Error] Invalid Optimizer object pointer.")

    def UsesDevicePath(self):
        return self.ctx is not None

    def Initialize(self):
        """SVGD.hpp:268-296: model, kernel and optimizer initialisation."""
        self.model_.Initialize()
        self.kernel_.Initialize()
        self.optimizer_.Initialize()
        self.logs_ = []
        self._initialized = True
        c = self.ctx
        if c is None:
            return
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
        if self.ctx is None:
            for it in range(self.num_iterations_):
                self._host_step(it)
            self._write_logs()
            return
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
                if _builtin_grad(self.model_):
                    self.model_.log_model_grad_ptr(c.x_host_ptr, nr, c.g_host_ptr)
                elif nr > 0:
                    c.g_host[:nr] = self.model_.log_model_grad(c.x_host[:nr])
                c.check(c.lib.svgd_finish_step(c.h, c.g_host_ptr))
            else:
                # logging re-evaluates K at X_t from the host buffers, which
                # only the split begin / finish calls fill (the pipelined step
                # may take X_t from its own mirror)
                c.step_with_model(self.model_, hessian=hess, pipelined=not self.log_)
            if self.log_:
                self._log_device_step(len(self.logs_))
        X = c.get_particles()
        self.coord_matrix_[...] = X.T
        self._write_logs()

    # -- generic kernel: the reference's ComputePhi on the host (SVGD.hpp:373-454)
    def _host_step(self, it):
        X = self.coord_matrix_  # (d, n), updated in place like *coord_matrix_ptr_
        d, n = X.shape
        self.model_.Step()
        self.kernel_.Step()
        P = np.ascontiguousarray(X.T)
        G = self.model_.log_model_grad(P)  # (n, d)
        K = np.empty((n, n))
        Kg = np.empty((d * n, n))
        k = self.kernel_
        for i in range(n):
            k.UpdateLocation(P[i])
            k.Initialize()
            for j in range(n):
                K[j, i] = k.EvaluateKernel(P[j])  # k(x_j, x_i)
                Kg[j * d:(j + 1) * d, i] = k.EvaluateKernelGrad(P[j])
        phi = (1.0 / n) * (G.T @ K + Kg.reshape(n, d, n).sum(axis=0))
        X += self.optimizer_.Step(phi)
        if self.bounds_ is not None:
            lo, hi = self.bounds_
            X[...] = np.maximum(np.minimum(X, hi[:, None]), lo[:, None])
        if self.log_:
            self._log(it, G.T, K, Kg, X)

    def _log_device_step(self, it):
        c = self.ctx
        n = self.coord_matrix_.shape[1]
        nr = c.row1 - c.row0
        P, G = c.x_host[:nr].copy(), c.g_host[:nr].copy()  # X_t and grad log p(X_t) of the step
        d = P.shape[1]
        M = c.get_scale_matrix()
        K = np.empty((n, n))
        Kg = np.empty((d * n, n))
        for i in range(n):
            diff = P - P[i]  # x_j - x_i
            Md = diff @ M.T
            kv = np.exp(-np.einsum("jk,jk->j", diff, Md))
            K[:, i] = kv
            Kg[:, i] = (-2.0 * Md * kv[:, None]).reshape(-1)
        self._log(it, G.T, K, Kg, c.get_particles().T)

    def _log(self, it, G, K, Kg, X):
        def fmt(A):
            prec = self.log_precision_ or 6
            cells = [[f"{v:.{prec}g}" for v in row] for row in np.atleast_2d(A)]
            w = max(len(c) for row in cells for c in row)
            return "\n".join(" ".join(c.rjust(w) for c in row) for row in cells)
        self.logs_.append(f"========== Step {it + 1} ==========\nLogModelGrad=\n{fmt(G)}\n\nKernel=\n{fmt(K)}"
                          f"\n\nKernelGrad=\n{fmt(Kg)}\n\nCoordMat=\n{fmt(X)}\n\n")

    def _write_logs(self):
        if not self.log_:
            return
        try:
            with open(self.log_path_, "w") as f:
                f.write("".join(self.logs_))
        except OSError:
            raise RuntimeError(PREFIX + f"[Runtime Error] Cannot open {self.log_path_} for writing.")

    def UpdateKernelParameters(self, params):  # SVGD.hpp:304-320
        self.kernel_.UpdateParameters(params)
        self.kernel_.Initialize()
        if self.ctx is not None:
            self.Initialize()

    def UpdateModelParameters(self, params):  # SVGD.hpp:328-332
        self.model_.UpdateParameters(params)
        self.model_.Initialize()
