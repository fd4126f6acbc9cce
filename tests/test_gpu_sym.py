"""Symmetric phi pass (k_phi_sym: the default for one rank at d <= 8; SVGD_PHI_SYM=1
forces it here, =0 selects the row stream): parity with the CPU oracle
through the C ABI.  GPU only.

Each unordered pair's kernel value feeds both particles (SVGD.hpp:453 with
K_ij = K_ji), so phi_i is assembled from row and column partials in a fixed
order -- a different summation order from the row stream, same tolerance:

  * phi_hat from identical (X, G, a):   max-abs <= 1e-10 (north star)
  * against the row stream on the same inputs: max-abs <= 1e-12
  * repeated launches:                  bit-identical (deterministic order)
  * a step (median + phi + Adam):       positions <= 1e-9 vs the oracle step
  * far outliers (a log2e max|xc|^2 > 300): the record prep's flag hands the
    step to the row stream, same bar
"""
import numpy as np
import pytest

import svgdcpp_amd as S
from svgdcpp_amd import _capi as C

pytestmark = pytest.mark.gpu

PHI_TOL = 1e-10


@pytest.fixture(params=["1", "2"])
def sym_env(monkeypatch, request):
    """1: the one-rank pass (k_sym_finish forms phi); 2: the sharded form at
    one rank (every particle's sums, the exchange's call site with no
    communicator, k_sym_apply) -- including the row-stream hand-over, whose
    partials the finish / apply sum."""
    monkeypatch.setenv("SVGD_PHI_SYM", request.param)


def _ctx(X, **kw):
    n, d = X.shape
    c = S.Context(d, n, **kw)
    c.set_particles(X)
    return c


# n around the work-group block B = 512 R (R = 8, 8, 6, 5, 4, 3, 3, 3 rows per
# lane for d = 1..8: B = 4096, 4096, 3072, 2560, 2048, 1536, 1536, 1536): a
# single partial block, exact multiples, ragged tails, and several blocks
# (odd and even block counts of the tile plan)
@pytest.mark.parametrize("n,d", [(1, 2), (2, 1), (5, 8), (64, 3), (300, 8), (1536, 8), (1537, 8),
                                 (3072, 8), (3100, 8), (4700, 8), (6200, 8), (700, 2), (4096, 2),
                                 (5000, 2), (9000, 2), (13000, 2), (3000, 1), (9000, 1), (1500, 3),
                                 (7000, 3), (1100, 4), (6000, 4), (900, 5), (5000, 5), (800, 6),
                                 (3500, 6), (700, 7), (3500, 7)])
def test_sym_phi_matches_oracle(oracle, sym_env, n, d):
    X = oracle.splitmix((n, d), 2.0, 300 + n + d)
    G = oracle.splitmix((n, d), 1.0, 400 + n + d)
    a = 0.37
    c = _ctx(X)
    ph = c.phi(G, a)
    ref = oracle.phi(X, G, a)
    assert np.max(np.abs(ph - ref)) <= PHI_TOL
    c.close()


@pytest.mark.parametrize("n,d", [(2100, 8), (4000, 2)])
def test_sym_matches_row_stream_and_is_deterministic(oracle, monkeypatch, n, d):
    X = oracle.splitmix((n, d), 3.0, 7 + d)
    G = oracle.splitmix((n, d), 1.0, 8 + d)
    a = 0.21
    monkeypatch.setenv("SVGD_PHI_SYM", "0")
    row = _ctx(X).phi(G, a)
    monkeypatch.setenv("SVGD_PHI_SYM", "1")
    c = _ctx(X)
    p1 = c.phi(G, a)
    p2 = c.phi(G, a)
    assert np.array_equal(p1, p2)
    assert np.max(np.abs(p1 - row)) <= 1e-12
    c.close()


def test_sym_far_outliers_fall_back_to_row_stream(oracle, sym_env):
    """a log2e max|xc|^2 >> 300: the symmetric form would leave its exponent
    range, the record prep's flag skips it and the row stream (plain form)
    computes phi -- same bar against the oracle."""
    n, d = 1200, 8
    X = oracle.splitmix((n, d), 1.0, 91)
    X[:3] += 40.0
    G = oracle.splitmix((n, d), 1.0, 92)
    a = 0.5
    ref = oracle.phi(X, G, a)
    ph = _ctx(X).phi(G, a)
    assert np.max(np.abs(ph - ref)) <= PHI_TOL


@pytest.mark.parametrize("opt", ["adam", "adagrad", "rmsprop"])
@pytest.mark.parametrize("bounded", [False, True])
def test_sym_steps_match_oracle(oracle, sym_env, opt, bounded):
    """Median scale + symmetric phi + optimizer (+ the bounds clamp,
    SVGD.hpp:393-399), several steps, each step against the oracle step from
    the same X_t (scale rel <= 1e-12).  The finish (k_sym_finish) and the
    sharded apply (k_sym_apply) run the optimizer epilogue themselves."""
    n, d, k = 3000, 8, 4
    X = oracle.splitmix((n, d), 3.0, 0x5EED)
    mus = oracle.splitmix((k, d), 3.0, 0x5EEE)
    covs = np.stack([np.eye(d) * (1.0 + 0.25 * q) for q in range(k)])
    model = S.GaussianSum(list(mus), list(covs))
    c = _ctx(X)
    if opt == "adam":
        c.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999, 1e-8)
        ref_opt = oracle.Adam((n, d), 0.1, 0.9, 0.999)
    elif opt == "adagrad":
        c.set_optimizer(C.SVGD_OPT_ADAGRAD, 0.1, 0.0, 0.0, 1e-8)
        ref_opt = oracle.AdaGrad((n, d), 0.1)
    else:
        c.set_optimizer(C.SVGD_OPT_RMSPROP, 0.1, 0.9, 0.0, 1e-8)
        ref_opt = oracle.RMSProp((n, d), 0.1, 0.9)
    lo = up = None
    if bounded:  # tight enough that every step clamps some coordinates
        lo, up = -np.full(d, 2.8), np.full(d, 2.5)
        c.set_bounds(lo, up)
    assert c.phi_kernel_name().startswith("k_phi_sym")
    Xt = X.copy()
    clamped = 0
    for _ in range(4):
        c.step_with_model(model)
        a_dev, _, _ = c.last_scale()
        a_ref, _ = oracle.median_scale(Xt)
        assert a_dev == pytest.approx(a_ref, rel=1e-12)
        G = oracle.logp_grad_gmm(Xt, mus, covs)
        Xr = Xt.copy()
        oracle.apply_update(Xr, ref_opt.step(oracle.phi(Xt, G, a_dev)), lo, up)
        X1 = c.get_particles()
        assert np.max(np.abs(X1 - Xr)) <= 1e-9
        if bounded:
            assert X1.min() >= -2.8 and X1.max() <= 2.5
            clamped += int(np.sum(X1 == -2.8) + np.sum(X1 == 2.5))
        Xt = X1
    assert not bounded or clamped > 0
    c.close()


def test_sym_full_size_rows_match_oracle(oracle, sym_env):
    """cfg3 size (N = 65536, d = 8): sampled rows -- both ends and a block
    straddling several work-group row blocks and tiles -- against the oracle's
    rows of the same phi."""
    n, d = 65536, 8
    X = oracle.splitmix((n, d), 3.0, 0x5EED)
    G = oracle.splitmix((n, d), 1.0, 77)
    c = _ctx(X)
    a, _ = c.median_scale()
    ph = c.phi(G, a)
    for r0, r1 in ((0, 128), (30000, 30800), (n - 128, n)):
        ref = oracle.phi(X, G, a, rows=(r0, r1))
        assert np.max(np.abs(ph[r0:r1] - ref)) <= PHI_TOL, (r0, r1)
    c.close()


def test_sym_context_takes_row_stream_for_matrix_scale(oracle, sym_env):
    """A context planned for the symmetric pass: an isotropic phi (the
    pass), then a full-matrix scale (the folded form needs an isotropic a:
    the row stream with the matrix records runs), then isotropic again --
    each against the oracle."""
    n, d = 2000, 8
    X = oracle.splitmix((n, d), 2.0, 501)
    G = oracle.splitmix((n, d), 1.0, 502)
    A = np.random.default_rng(3).standard_normal((d, d)) * 0.4
    M = (A @ A.T + 0.3 * np.eye(d)) / d
    a = 0.37
    c = _ctx(X)
    assert c.phi_kernel_name().startswith("k_phi_sym")
    ref = oracle.phi(X, G, a)
    assert np.max(np.abs(c.phi(G, a) - ref)) <= PHI_TOL
    c.set_scale_matrix(M)
    assert np.max(np.abs(c.phi(G, 0.0) - oracle.phi_matrix(X, G, M))) <= PHI_TOL
    c.set_scale(C.SVGD_SCALE_MEDIAN)
    assert np.max(np.abs(c.phi(G, a) - ref)) <= PHI_TOL
    c.close()
