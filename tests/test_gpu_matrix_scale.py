"""Full-matrix kernel scale on the device: ScaleMethod::Hessian
(GaussianRBFKernel.hpp:189-210, M = sum_i -hess log p(x_i) / (2 d N)) and a
fixed symmetric positive-definite M (the Constant extension with a full
matrix).  Parity against the oracle's restatement (oracle.phi_matrix,
oracle.hessian_scale), which is checked on the CPU against finite
differences of the model gradient and against the isotropic oracle
(tests/test_oracle.py).  Tolerances: phi max-abs 1e-10 (north star), the
scale matrix rel 1e-12, per-step positions 1e-9."""
import numpy as np
import pytest

import svgdcpp_amd as S
from svgdcpp_amd import _capi as C

pytestmark = pytest.mark.gpu


def _spd(d, seed):
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((d, d)) * 0.4
    return A @ A.T + np.eye(d) * 0.3


@pytest.mark.parametrize("n,d", [(500, 2), (1500, 8), (700, 13), (600, 24)])
def test_phi_fixed_matrix_scale(oracle, n, d):
    X = oracle.splitmix((n, d), 2.0, 11 + d)
    G = oracle.splitmix((n, d), 1.0, 12 + d)
    M = _spd(d, d) / d
    c = S.Context(d, n)
    c.set_particles(X)
    c.set_scale_matrix(M)
    ph = c.phi(G, 0.0)
    ref = oracle.phi_matrix(X, G, M)
    assert np.max(np.abs(ph - ref)) <= 1e-10
    np.testing.assert_allclose(c.get_scale_matrix(), M, rtol=1e-15, atol=0)


@pytest.mark.parametrize("d,k", [(3, 2), (8, 4)])
def test_hessian_scale_step_matches_oracle(oracle, d, k):
    n = 1200
    X = oracle.splitmix((n, d), 3.0, 31)
    mus = oracle.splitmix((k, d), 2.0, 32)
    covs = np.stack([_spd(d, 40 + i) + np.eye(d) for i in range(k)])
    model = S.GaussianSum(list(mus), list(covs))
    c = S.Context(d, n)
    c.set_particles(X)
    c.set_optimizer(C.SVGD_OPT_ADAM, 0.05, 0.9, 0.999, 1e-8)
    c.set_scale(C.SVGD_SCALE_HESSIAN, 0.0)
    o_opt = oracle.Adam((n, d), 0.05, 0.9, 0.999)
    for _ in range(3):
        Xt = c.get_particles()
        M = oracle.hessian_scale(Xt, mus, covs)
        G = oracle.logp_grad_gmm(Xt, mus, covs)
        ph = oracle.phi_matrix(Xt, G, M)
        c.step_with_model(model, hessian=True)
        np.testing.assert_allclose(c.get_scale_matrix(), M, rtol=1e-12, atol=1e-15)
        Xref = Xt.copy()
        oracle.apply_update(Xref, o_opt.step(ph))
        assert np.max(np.abs(c.get_particles() - Xref)) <= 1e-9


def test_hessian_scale_errors(oracle):
    n, d = 50, 2
    c = S.Context(d, n)
    c.set_particles(oracle.splitmix((n, d), 1.0, 3))
    c.set_optimizer(C.SVGD_OPT_ADAM, 0.05, 0.9, 0.999, 1e-8)
    c.set_scale(C.SVGD_SCALE_HESSIAN, 0.0)
    model = S.GaussianSum([np.zeros(d)], [np.eye(d)])
    with pytest.raises(S.UnsetException):
        c.step_with_model(model)  # no Hessian sum supplied
    with pytest.raises(ValueError):
        c.set_scale_matrix(np.array([[1.0, 0.5], [0.4, 1.0]]))  # not symmetric
    # an indefinite M on the MFMA tile path (d > 16) fails loudly before phi
    d3 = 24
    c3 = S.Context(d3, n)
    c3.set_particles(oracle.splitmix((n, d3), 1.0, 3))
    M3 = np.eye(d3)
    M3[0, 0] = -0.5
    c3.set_scale_matrix(M3)
    with pytest.raises(S.DeviceError):
        c3.phi(np.zeros((n, d3)), 0.0)


def _indefinite(d, seed):
    rng = np.random.default_rng(seed)
    Q, _ = np.linalg.qr(rng.standard_normal((d, d)))
    lam = rng.uniform(0.2, 1.0, d) * np.where(np.arange(d) % 3 == 1, -0.3, 1.0)
    if d == 2:
        lam = np.array([0.8, -0.25])
    M = (Q * lam) @ Q.T
    return 0.5 * (M + M.T)  # exactly symmetric


@pytest.mark.parametrize("n,d", [(500, 2), (900, 5), (1500, 8), (700, 16)])
def test_phi_indefinite_matrix_scale(oracle, n, d):
    """GaussianRBFKernel.hpp:75-81 evaluates exp(-(x-x')^T M (x-x')) for any
    symmetric M; an indefinite M (e.g. a Hessian sum between mixture modes)
    is factored M = L S L^T by the Jacobi eigendecomposition on the row path."""
    X = oracle.splitmix((n, d), 1.0, 21 + d)
    G = oracle.splitmix((n, d), 1.0, 22 + d)
    M = _indefinite(d, d) * (0.5 / d)
    assert np.min(np.linalg.eigvalsh(M)) < 0
    c = S.Context(d, n)
    c.set_particles(X)
    c.set_scale_matrix(M)
    ph = c.phi(G, 0.0)
    ref = oracle.phi_matrix(X, G, M)
    assert np.max(np.abs(ph - ref)) <= 1e-10 * max(1.0, np.max(np.abs(ref)))
    np.testing.assert_allclose(c.get_scale_matrix(), M, rtol=1e-15, atol=0)
    c.close()


def test_svgd_class_hessian_scale(oracle):
    """The SVGD driver with GaussianRBFKernel(ScaleMethod.Hessian) vs the
    oracle loop (SVGD.hpp:373-400 with the Hessian scale each step)."""
    n, d, iters = 300, 2, 6
    mu, cov = np.array([-0.6871, 0.8010]), 5 * np.array([[0.2260, 0.1652], [0.1652, 0.6779]])
    X0 = oracle.splitmix((n, d), 3.0, 5)
    coord = np.ascontiguousarray(X0.T).copy()
    model = S.MultivariateNormal(mu, cov)
    kern = S.GaussianRBFKernel(coord, S.GaussianRBFKernel.ScaleMethod.Hessian, model)
    opt = S.Adam(d, n, 0.1, 0.9, 0.999)
    sv = S.SVGD(d, iters, coord, kern, model, opt)
    sv.Initialize()
    sv.Run()
    X = X0.copy()
    o_opt = oracle.Adam((n, d), 0.1, 0.9, 0.999)
    for _ in range(iters):
        M = oracle.hessian_scale(X, mu[None], cov[None])
        G = oracle.logp_grad_gmm(X, mu[None], cov[None])
        oracle.apply_update(X, o_opt.step(oracle.phi_matrix(X, G, M)))
    np.testing.assert_allclose(coord.T, X, rtol=0, atol=1e-9)
