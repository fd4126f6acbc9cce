"""ctypes wrapper around oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference's SVGD inner step (see svgd_oracle.c for
the per-function reference citations).  Imported only by tests/,
``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg, always as the
checker / baseline, never as the product path.

Arrays follow the reference layout: a d×n column-major Eigen matrix is a
C-contiguous numpy array of shape (n, d) (particle i = row i).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

_D = ctypes.POINTER(ctypes.c_double)
_L = ctypes.c_long


def build(force: bool = False) -> str:
    """Compile liboracle.so with the committed Makefile (gcc, OpenMP)."""
    if force or not os.path.exists(_LIB_PATH) or (
        os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "svgd_oracle.c"))
    ):
        subprocess.run(["make", "-C", _HERE, "-B" if force else "liboracle.so"], check=True,
                       stdout=subprocess.DEVNULL)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        l = ctypes.CDLL(_LIB_PATH)
        l.or_fill_eigen_random.argtypes = [_D, _L, ctypes.c_double, ctypes.c_uint]
        l.or_fill_splitmix.argtypes = [_D, _L, ctypes.c_double, ctypes.c_uint64]
        l.or_pairwise_dist_gram.argtypes = [_D, ctypes.c_int, _L, _D]
        l.or_median.argtypes = [_D, _L]
        l.or_median.restype = ctypes.c_double
        l.or_median_scale.argtypes = [_D, ctypes.c_int, _L, _D, _D]
        l.or_upper_sqdist_kth.argtypes = [_D, ctypes.c_int, _L, _L]
        l.or_upper_sqdist_kth.restype = ctypes.c_double
        l.or_phi_rows.argtypes = [_D, _D, ctypes.c_int, _L, ctypes.c_double, _L, _L, _D, _D, _D]
        l.or_adam.argtypes = [_D, _D, _D, _L, _L, ctypes.c_double, ctypes.c_double,
                              ctypes.c_double, ctypes.c_double, _D]
        l.or_adagrad.argtypes = [_D, _D, _L, ctypes.c_double, ctypes.c_double, _D]
        l.or_rmsprop.argtypes = [_D, _D, _L, ctypes.c_double, ctypes.c_double, ctypes.c_double, _D]
        l.or_apply_update.argtypes = [_D, _D, ctypes.c_int, _L, _D, _D]
        l.or_logp_grad_gmm.argtypes = [_D, ctypes.c_int, _L, ctypes.c_int, _D, _D, _D]
        l.or_median_rows_work.argtypes = [_D, ctypes.c_int, _L, _L, _L]
        l.or_median_rows_work.restype = ctypes.c_double
        l.or_num_threads.restype = ctypes.c_int
        l.or_set_threads.argtypes = [ctypes.c_int]
        l.or_upper_sqdist_counts.argtypes = [_D, ctypes.c_int, _L, _D, ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_longlong)]
        l.or_neg_hess_sum_gmm.argtypes = [_D, ctypes.c_int, _L, ctypes.c_int, _D, _D, _D]
        l.or_phi_matrix_rows.argtypes = [_D, _D, ctypes.c_int, _L, _D, _L, _L, _D]
        _lib = l
    return _lib


def _p(a):
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_D)


def eigen_random(d: int, n: int, scale: float = 1.0, seed: int = 1) -> np.ndarray:
    """scale * Eigen::MatrixXd::Random(d, n) in a fresh process (glibc rand, srand(seed))."""
    x = np.empty((n, d), dtype=np.float64)
    lib().or_fill_eigen_random(_p(x), n * d, scale, seed)
    return x


def splitmix(count_shape, scale: float = 1.0, seed: int = 0x5EED) -> np.ndarray:
    x = np.empty(count_shape, dtype=np.float64)
    lib().or_fill_splitmix(_p(x), x.size, scale, seed)
    return x


def pairwise_dist_gram(X: np.ndarray) -> np.ndarray:
    n, d = X.shape
    out = np.empty((n, n), dtype=np.float64)
    lib().or_pairwise_dist_gram(_p(np.ascontiguousarray(X)), d, n, _p(out))
    return out


def median_scale(X: np.ndarray):
    """(a, med) of GaussianRBFKernel::ComputeScale (Median)."""
    n, d = X.shape
    a = ctypes.c_double()
    m = ctypes.c_double()
    lib().or_median_scale(_p(np.ascontiguousarray(X)), d, n, ctypes.byref(a), ctypes.byref(m))
    return a.value, m.value


def upper_sqdist_kth(X: np.ndarray, k: int) -> float:
    n, d = X.shape
    return lib().or_upper_sqdist_kth(_p(np.ascontiguousarray(X)), d, n, k)


def upper_sqdist_counts(X: np.ndarray, thresholds):
    """For each threshold t: #pairs i<j with direct-form D^2 < t (one streamed pass)."""
    n, d = X.shape
    t = np.ascontiguousarray(thresholds, dtype=np.float64)
    out = (ctypes.c_longlong * len(t))()
    lib().or_upper_sqdist_counts(_p(np.ascontiguousarray(X)), d, n, _p(t), len(t), out)
    return [int(v) for v in out]


def phi(X, G, a, rows=None, materialise=False):
    """phi_hat (n×d) for rows [i0, i1); optionally K (n×n, K[i, j] = k(x_j, x_i))
    and Kg (n×n×d, Kg[i, j] = ∇_{x_j} k(x_j, x_i))."""
    n, d = X.shape
    i0, i1 = rows if rows is not None else (0, n)
    out = np.empty((i1 - i0, d), dtype=np.float64)
    K = np.empty((n, n)) if materialise else None
    Kg = np.empty((n, n, d)) if materialise else None
    lib().or_phi_rows(_p(np.ascontiguousarray(X)), _p(np.ascontiguousarray(G)), d, n, float(a),
                      i0, i1, _p(out), _p(K), _p(Kg))
    return (out, K, Kg) if materialise else out


class Adam:
    """Adam.hpp:33-96."""

    def __init__(self, shape, lr, b1, b2, eps=1e-8):
        if b1 >= 1.0 or b1 < 0.0 or b2 >= 1.0 or b2 < 0.0:
            raise ValueError("SVGDCpp: [Argument Error] Invalid value for decay parameter beta.")
        self.m = np.zeros(shape)
        self.v = np.zeros(shape)
        self.t = 0
        self.lr, self.b1, self.b2, self.eps = lr, b1, b2, eps

    def step(self, g):
        self.t += 1
        g = np.ascontiguousarray(g, dtype=np.float64)
        out = np.empty_like(g)
        lib().or_adam(_p(self.m), _p(self.v), _p(g), g.size, self.t, self.lr, self.b1, self.b2,
                      self.eps, _p(out))
        return out


class AdaGrad:
    """AdaGrad.hpp:33-65."""

    def __init__(self, shape, lr, eps=1e-8):
        self.v = np.zeros(shape)
        self.lr, self.eps = lr, eps

    def step(self, g):
        g = np.ascontiguousarray(g, dtype=np.float64)
        out = np.empty_like(g)
        lib().or_adagrad(_p(self.v), _p(g), g.size, self.lr, self.eps, _p(out))
        return out


class RMSProp:
    """RMSProp.hpp:32-74."""

    def __init__(self, shape, lr, beta, eps=1e-8):
        if beta > 1.0 or beta < 0.0:
            raise ValueError("SVGDCpp: [Argument Error] Invalid value for decay parameter beta.")
        self.v = np.zeros(shape)
        self.lr, self.beta, self.eps = lr, beta, eps

    def step(self, g):
        g = np.ascontiguousarray(g, dtype=np.float64)
        out = np.empty_like(g)
        lib().or_rmsprop(_p(self.v), _p(g), g.size, self.lr, self.beta, self.eps, _p(out))
        return out


def apply_update(X, delta, lower=None, upper=None):
    """SVGD.hpp:393-399, in place on X."""
    n, d = X.shape
    lo = None if lower is None else np.ascontiguousarray(lower, dtype=np.float64)
    up = None if upper is None else np.ascontiguousarray(upper, dtype=np.float64)
    lib().or_apply_update(_p(X), _p(np.ascontiguousarray(delta)), d, n, _p(lo), _p(up))


def logp_grad_gmm(X, mus, covs):
    """∇ log Σ_c exp(-½ q_c(x)) (unweighted, unnormalised); mus (k,d), covs (k,d,d)."""
    n, d = X.shape
    mus = np.ascontiguousarray(mus, dtype=np.float64).reshape(-1, d)
    covs = np.ascontiguousarray(covs, dtype=np.float64).reshape(-1, d, d)
    G = np.empty((n, d))
    lib().or_logp_grad_gmm(_p(np.ascontiguousarray(X)), d, n, mus.shape[0], _p(mus), _p(covs), _p(G))
    return G


def median_rows_work(X, i0, i1) -> float:
    """Median work of rows [i0, i1) (their share of the distinct pairs) -- for
    timing a bounded sample of a large step."""
    n, d = X.shape
    return lib().or_median_rows_work(_p(np.ascontiguousarray(X)), d, n, i0, i1)


def neg_hess_sum_gmm(X, mus, covs):
    """-sum_i hess log p(x_i) for the Gaussian-sum model (d x d)."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    n, d = X.shape
    mus = np.ascontiguousarray(mus, dtype=np.float64)
    covs = np.ascontiguousarray(covs, dtype=np.float64)
    H = np.empty((d, d))
    lib().or_neg_hess_sum_gmm(_p(X), d, n, mus.shape[0], _p(mus), _p(covs), _p(H))
    return H


def hessian_scale(X, mus, covs):
    """GaussianRBFKernel.hpp:189-210: M = sum_i -hess log p(x_i) / (2 d N)."""
    n, d = np.asarray(X).shape
    return neg_hess_sum_gmm(X, mus, covs) / (2.0 * d * n)


def phi_matrix(X, G, M, rows=None):
    """phi_hat with a full kernel scale matrix M (rows [i0, i1))."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    n, d = X.shape
    i0, i1 = rows if rows is not None else (0, n)
    out = np.empty((i1 - i0, d))
    M = np.ascontiguousarray(M, dtype=np.float64)
    lib().or_phi_matrix_rows(_p(X), _p(np.ascontiguousarray(G, dtype=np.float64)), d, n, _p(M),
                             i0, i1, _p(out))
    return out


def num_threads() -> int:
    return lib().or_num_threads()


def set_threads(n: int) -> None:
    lib().or_set_threads(int(n))


def run_svgd(X0, grad_fn, steps, optimizer, scale="median", lower=None, upper=None):
    """SVGD::Run (SVGD.hpp:338-400) on the oracle: per step the scale from X_t
    (median, or a fixed float), phi_hat, optimizer increment, clamp.  Returns X."""
    X = np.array(X0, dtype=np.float64, copy=True)
    for _ in range(steps):
        a = median_scale(X)[0] if scale == "median" else float(scale)
        G = grad_fn(X)
        ph = phi(X, G, a)
        apply_update(X, optimizer.step(ph), lower, upper)
    return X
