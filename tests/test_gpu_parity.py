"""Parity of the HIP path (through the C ABI) with the CPU oracle.  GPU only.

Tolerances (fp64, north star: <= 1e-10 max-abs on phi_hat):
  * phi_hat from identical (X, G, a):            max-abs <= 1e-10 (observed ~1e-15)
  * median / scale a:                            rel <= 1e-12 (ulp-level: the device
    computes the Gram form on mean-centred coordinates, the oracle on raw ones)
  * median selection:                            BIT-EXACT against the exact order
    statistics of the device's own keys (svgd_debug_pair_keys)
  * optimizer + clamp on identical phi:          BIT-EXACT
  * 1000-iteration notebook trajectories:        the published 6 significant digits
"""
import json
import os

import numpy as np
import pytest

import svgdcpp_amd as S
from svgdcpp_amd import _capi as C

pytestmark = pytest.mark.gpu

PHI_TOL = 1e-10


def _ctx(X, **kw):
    n, d = X.shape
    c = S.Context(d, n, **kw)
    c.set_particles(X)
    return c


def _gmm(oracle, d, k, seed):
    mus = oracle.splitmix((k, d), 3.0, seed)
    covs = np.stack([np.eye(d) * (1.0 + 0.25 * c) for c in range(k)])
    return mus, covs


@pytest.mark.parametrize("name", ["n256_d2", "n1000_d8", "n300_d64", "n77_d3"])
def test_phi_and_scale_match_golden(golden_dir, name):
    z = np.load(os.path.join(golden_dir, f"phi_{name}.npz"))
    c = _ctx(z["X"])
    a, med = c.median_scale()
    assert med == pytest.approx(float(z["med"]), rel=1e-12)
    assert a == pytest.approx(float(z["a"]), rel=1e-12)
    ph = c.phi(z["G"], float(z["a"]))
    assert np.max(np.abs(ph - z["phi"])) <= PHI_TOL


@pytest.mark.parametrize("n,d", [(1, 2), (2, 1), (3, 3), (63, 2), (64, 4), (65, 5), (130, 7),
                                 (200, 8), (129, 12), (97, 13), (70, 16), (50, 17), (40, 32),
                                 (33, 33), (31, 63), (20, 64)])
def test_phi_random_shapes(oracle, n, d):
    X = oracle.splitmix((n, d), 2.0, 100 + n + d)
    G = oracle.splitmix((n, d), 1.0, 200 + n + d)
    a = 0.37
    c = _ctx(X)
    ph = c.phi(G, a)
    ref = oracle.phi(X, G, a)
    assert np.max(np.abs(ph - ref)) <= PHI_TOL


@pytest.mark.parametrize("n,d", [(1, 2), (5, 8), (200, 8), (1000, 8), (2049, 8), (4000, 2),
                                 (777, 3), (130, 12), (70, 16)])
def test_phi_row_kernel(oracle, monkeypatch, n, d):
    """The row stream (8 waves splitting one row group's columns, their sums
    added in LDS in wave order; SVGD_PHI_SYM=0 -- one rank at d <= 8 takes
    the symmetric pass by default, tests/test_gpu_sym.py) against the oracle,
    and deterministic.  (The 4-wave kernel it replaced serves the full-matrix
    scales and is covered by tests/test_gpu_matrix_scale.py.)"""
    monkeypatch.setenv("SVGD_PHI_SYM", "0")
    X = oracle.splitmix((n, d), 2.0, 500 + n + d)
    G = oracle.splitmix((n, d), 1.0, 600 + n + d)
    a = 0.29
    ref = oracle.phi(X, G, a)
    c = _ctx(X)
    assert c.phi_kernel_name().startswith("k_phi_rows<%d, %d, 8, 8192, 8>" % (d, 4 if d <= 8 else 2))
    out = c.phi(G, a)
    assert np.array_equal(out, c.phi(G, a))  # deterministic
    c.close()
    assert np.max(np.abs(out - ref)) <= PHI_TOL


@pytest.mark.parametrize("n,d", [(300, 32), (1111, 32), (1111, 48), (300, 64), (1111, 64), (1111, 17),
                                 (1111, 33), (1111, 63), (129, 64)])
def test_phi_tile_kernel_variants(oracle, monkeypatch, n, d):
    """The fp64 tile kernel (d > 16, k_phi<double>: 8-wave blocks of 128 rows,
    j-major X_J in LDS): with d = 16 NCB its row sums run on the VALU
    (SVGD_PHI_S1V, default) or through a V column of ones (=0).  Ragged n
    leaves a partial last row block and padded columns j >= n, which the VALU
    sums must mask.  Both against the oracle; against each other only the
    summation order of s1 differs."""
    X = oracle.splitmix((n, d), 2.0, 700 + n + d)
    G = oracle.splitmix((n, d), 1.0, 800 + n + d)
    a = 0.05
    ref = oracle.phi(X, G, a)
    out = {}
    for v in ("1", "0"):
        monkeypatch.setenv("SVGD_PHI_S1V", v)
        c = _ctx(X)
        out[v] = c.phi(G, a)
        name = c.phi_kernel_name()
        c.close()
        assert name.startswith("k_phi<double"), name
        assert name.endswith("true>") == (v == "1" and d % 16 == 0), name
        assert np.max(np.abs(out[v] - ref)) <= PHI_TOL, (v, name)
    assert np.max(np.abs(out["1"] - out["0"])) <= 1e-12


def test_phi_far_from_origin(oracle):
    """Translation: particles around 1e3 (mean-centring keeps the x_i*sum K -
    sum K x_j assembly accurate)."""
    n, d = 300, 4
    X = 1000.0 + oracle.splitmix((n, d), 1.0, 9)
    G = oracle.splitmix((n, d), 1.0, 10)
    a = 1.3
    ref = oracle.phi(X, G, a)
    ph = _ctx(X).phi(G, a)
    assert np.max(np.abs(ph - ref)) <= PHI_TOL


@pytest.mark.parametrize("d", [2, 8])
def test_phi_outliers_mixed_fold(oracle, d):
    """A few particles far out (a log2e max|x_i - mean|^2 >> 300): the whole
    launch takes k_phi_rows' plain form, whose exponent is clamped to
    +-1000 x 4096 (pairs with the outliers lie far beyond it: K ~ 2^-9000
    becomes 2^-1000); it agrees with the oracle."""
    n = 1500
    X = oracle.splitmix((n, d), 1.0, 77 + d)
    X[[5, 700, 1499]] += 40.0
    G = oracle.splitmix((n, d), 1.0, 78 + d)
    a = 2.0
    ref = oracle.phi(X, G, a)
    ph = _ctx(X).phi(G, a)
    assert np.max(np.abs(ph - ref)) <= PHI_TOL


@pytest.mark.parametrize("y", [150.0, 299.0, 301.0, 2000.0])
@pytest.mark.parametrize("d", [2, 8])
def test_phi_fold_exponent_bound(oracle, d, y):
    """k_phi_rows folds the row term and scales 2^q T[m] by an integer add to
    the exponent field (no clamp) only while y = a log2e max|xc|^2 <= 300
    keeps every folded exponent above -1001; one far particle puts y just
    either side of the bound (and far beyond it).  A wrapped exponent would
    show up as huge phi values; every case matches the oracle."""
    n = 1200
    X = oracle.splitmix((n, d), 1.0, 31 + d)
    X[17] += 6.0
    G = oracle.splitmix((n, d), 1.0, 32 + d)
    xc = X - X.mean(axis=0)
    a = y / (np.log2(np.e) * np.max(np.sum(xc * xc, axis=1)))
    ref = oracle.phi(X, G, a)
    ph = _ctx(X).phi(G, a)
    assert np.max(np.abs(ph - ref)) <= PHI_TOL


@pytest.mark.parametrize("n", [2, 3, 4, 5, 8, 9, 64, 65, 127, 400, 777])
def test_median_exact_selection_direct(oracle, n):
    d = 3
    X = oracle.splitmix((n, d), 1.0, 3 * n)
    c = _ctx(X)
    a, med = c.median_scale()
    keys = np.empty(n * (n - 1) // 2)
    c.check(c.lib.svgd_debug_pair_keys(c.h, C.dptr(keys), keys.size))
    # device keys agree with the direct-form distances to rounding
    iu = np.triu_indices(n, 1)
    ref_keys = ((X[iu[0]] - X[iu[1]]) ** 2).sum(-1)
    np.testing.assert_allclose(keys, ref_keys, rtol=1e-12, atol=1e-13)
    # exact order statistics of the device's own keys
    u = np.sort(keys)
    tot = n * n

    def at(k):
        return 0.0 if k < n else np.sqrt(u[(k - n) // 2])
    exp = (at(tot // 2 - 1) + at(tot // 2)) / 2 if tot % 2 == 0 else at(tot // 2)
    assert med == exp  # bit-exact selection
    assert med == pytest.approx(oracle.median_scale(X)[1], rel=1e-12)
    assert a == pytest.approx(np.log(n) / (exp * exp), rel=1e-15)
    assert c.last_scale()[2] == C.SVGD_MEDIAN_DIRECT


def _median_with_tuning(X, direct_max, sample, cap):
    c = _ctx(X)
    c.check(c.lib.svgd_set_median_tuning(c.h, direct_max, sample, cap))
    a, med = c.median_scale()
    return c, a, med


@pytest.mark.parametrize("n,d", [(700, 5), (1501, 5), (1300, 40)])
def test_median_bracket_path_exact(oracle, n, d):
    """d = 40 runs the MFMA tile path, whose bracket comes from sampled 64 x 64 tiles."""
    X = oracle.splitmix((n, d), 1.0, n)
    ref_c = _ctx(X)
    a0, m0 = ref_c.median_scale()  # direct path
    c, a, med = _median_with_tuning(X, 0, 1 << 14, -1)
    assert c.last_scale()[2] in (C.SVGD_MEDIAN_BRACKET, C.SVGD_MEDIAN_REBRACKET)
    assert med == m0 and a == a0


@pytest.mark.parametrize("n,d,sample", [(700, 5, 1 << 14), (1501, 5, 1 << 14), (1300, 40, 1 << 14),
                                         (2100, 3, 1 << 18), (900, 4, 1 << 10)])
def test_median_bucket_select_matches_digit_passes(oracle, monkeypatch, n, d, sample):
    """The bucket select (selected key-range buckets compacted and selected in
    one work-group) and the per-digit radix passes pick the same keys."""
    X = oracle.splitmix((n, d), 1.0, 3 * n + d)
    res = []
    for cap in ("16384", "0"):  # default path, then the digit passes only
        monkeypatch.setenv("SVGD_BUCKET_CAP", cap)
        c, a, med = _median_with_tuning(X, 0, sample, -1)
        assert c.last_scale()[2] in (C.SVGD_MEDIAN_BRACKET, C.SVGD_MEDIAN_REBRACKET)
        res.append((a, med))
    assert res[0] == res[1]
    ref_a, ref_med = oracle.median_scale(X)
    assert res[0][1] == pytest.approx(ref_med, rel=1e-12)


def test_median_bucket_select_ties(oracle, monkeypatch):
    """Heavy ties inside the selected bucket (5 distinct points)."""
    base = oracle.splitmix((5, 3), 1.0, 11)
    X = np.repeat(base, 60, axis=0)
    out = []
    for cap in ("16384", "0"):
        monkeypatch.setenv("SVGD_BUCKET_CAP", cap)
        c, a, med = _median_with_tuning(X, 0, 1 << 12, -1)
        out.append(med)
    assert out[0] == out[1]
    assert out[0] == pytest.approx(oracle.median_scale(X)[1], rel=1e-12)


@pytest.mark.parametrize("d", [5, 40])
def test_median_rebracket_path_exact(oracle, monkeypatch, d):
    """A bracket of ~0 sample-quantile sigmas (SVGD_MEDIAN_SIGMA=0) misses the
    order statistics most of the time: the library brackets again from the same
    sample at 8 sigma and repeats the collect pass.  Every outcome stays exact;
    at least one of the seeds must take the re-bracket path."""
    monkeypatch.setenv("SVGD_MEDIAN_SIGMA", "0")
    paths = []
    for seed in range(6):
        n = 1200 + 37 * seed
        X = oracle.splitmix((n, d), 1.0, 100 + seed)
        a0, m0 = _ctx(X).median_scale()  # direct path
        c, a, med = _median_with_tuning(X, 0, 1 << 14, -1)
        paths.append(c.last_scale()[2])
        assert med == m0 and a == a0, (seed, paths[-1])
    assert C.SVGD_MEDIAN_REBRACKET in paths, paths


def test_step_rebracket_matches_normal_bracket(oracle, monkeypatch):
    """Full steps whose bracket misses (SVGD_MEDIAN_SIGMA=0: re-bracket + a
    second collect pass, or the radix fallback) give bit-identical particles
    to steps with the default bracket: the median is exact either way."""
    n, d = 6000, 8  # N^2/2 > 2^24 pairs: the bracket path
    mus, covs = _gmm(oracle, d, 4, 31)
    X0 = oracle.splitmix((n, d), 3.0, 32)
    out = []
    for sigma in (None, "0"):
        if sigma is None:
            monkeypatch.delenv("SVGD_MEDIAN_SIGMA", raising=False)
        else:
            monkeypatch.setenv("SVGD_MEDIAN_SIGMA", sigma)
        c = _ctx(X0)
        c.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999, 1e-8)
        paths = []
        for _ in range(3):
            c.step_with_model(S.GaussianSum(list(mus), list(covs)))
            paths.append(c.last_scale()[2])
        out.append((c.get_particles(), paths))
    assert all(p == C.SVGD_MEDIAN_BRACKET for p in out[0][1]), out[0][1]
    assert any(p in (C.SVGD_MEDIAN_REBRACKET, C.SVGD_MEDIAN_FALLBACK) for p in out[1][1]), out[1][1]
    np.testing.assert_array_equal(out[0][0], out[1][0])


def test_median_fallback_path_exact(oracle):
    n = 900
    X = oracle.splitmix((n, 4), 1.0, 42)
    a0, m0 = _ctx(X).median_scale()
    # a 1-key candidate capacity forces the overflow -> streamed radix select
    c, a, med = _median_with_tuning(X, 0, 1 << 12, 1)
    assert c.last_scale()[2] == C.SVGD_MEDIAN_FALLBACK
    assert med == m0 and a == a0


def test_median_ties_and_duplicates(oracle):
    """Many coincident particles: heavy ties and zero distances."""
    base = oracle.splitmix((5, 2), 1.0, 1)
    X = np.repeat(base, 40, axis=0)  # 200 particles, 5 distinct points
    c = _ctx(X)
    a, med = c.median_scale()
    assert med == pytest.approx(oracle.median_scale(X)[1], rel=1e-12)
    c2, a2, med2 = _median_with_tuning(X, 0, 1 << 10, -1)
    assert med2 == med


def _run_device(X0, model, iters, kind, params, scale=None, bounds=None):
    n, d = X0.shape
    c = _ctx(X0)
    c.set_optimizer(kind, *params)
    if bounds is not None:
        c.set_bounds(*bounds)
    if scale is not None:
        c.set_scale(C.SVGD_SCALE_FIXED, scale)
    for _ in range(iters):
        c.step_with_model(model)
    return c.get_particles()


@pytest.mark.parametrize("case", ["mvn", "gmm"])
def test_published_notebook_trajectory(oracle, golden_dir, case):
    with open(os.path.join(golden_dir, "notebooks.json")) as f:
        nb = json.load(f)[case]
    n, d = nb["n"], nb["d"]
    X0 = oracle.eigen_random(d, n, nb["init_scale"], nb["seed"])
    model = S.GaussianSum(nb["means"], nb["covs"])
    opt = nb["optimizer"]
    if opt["kind"] == "adam":
        X = _run_device(X0, model, nb["iters"], C.SVGD_OPT_ADAM,
                        (opt["lr"], opt["beta1"], opt["beta2"], 1e-8))
    else:
        X = _run_device(X0, model, nb["iters"], C.SVGD_OPT_ADAGRAD, (opt["lr"], 0.0, 0.0, 1e-8))
    np.testing.assert_allclose(X, np.array(nb["final"]), rtol=5e-6, atol=1e-6)


def test_reference_test_svgd_scenario(oracle, golden_dir):
    """tests/test_svgd.cpp: fixed exp(-|x-x'|^2), user model, Adam, bounds [-1,1]^2."""
    from golden.make_golden import test_svgd_model_grad

    class CosModel(S.Model):
        def __init__(self):
            super().__init__(2)

        def log_model_grad(self, X):
            return test_svgd_model_grad(np.asarray(X))

    with open(os.path.join(golden_dir, "test_svgd_n10.json")) as f:
        g = json.load(f)
    X0 = np.array(g["initial"])
    X = _run_device(X0, CosModel(), g["iters"], C.SVGD_OPT_ADAM, (0.1, 0.9, 0.999, 1e-8),
                    scale=1.0, bounds=(np.array(g["lower"]), np.array(g["upper"])))
    np.testing.assert_allclose(X, np.array(g["final"]), rtol=0, atol=1e-12)


@pytest.mark.parametrize("kind", ["adam", "adagrad", "rmsprop"])
def test_step_matches_oracle_per_step(oracle, kind):
    """Per-step parity on a GMM (n=333, d=6): each device step vs the oracle step
    started from the device's own X_t (so differences do not accumulate)."""
    n, d = 333, 6
    X = oracle.splitmix((n, d), 3.0, 5)
    mus, covs = _gmm(oracle, d, 3, 6)
    model = S.GaussianSum(list(mus), list(covs))
    c = _ctx(X)
    if kind == "adam":
        c.set_optimizer(C.SVGD_OPT_ADAM, 0.05, 0.9, 0.999, 1e-8)
        o_opt = oracle.Adam((n, d), 0.05, 0.9, 0.999)
    elif kind == "adagrad":
        c.set_optimizer(C.SVGD_OPT_ADAGRAD, 0.05, 0.0, 0.0, 1e-8)
        o_opt = oracle.AdaGrad((n, d), 0.05)
    else:
        c.set_optimizer(C.SVGD_OPT_RMSPROP, 0.05, 0.9, 0.0, 1e-8)
        o_opt = oracle.RMSProp((n, d), 0.05, 0.9)
    lo, up = -np.full(d, 2.5), np.full(d, 2.5)
    c.set_bounds(lo, up)
    for _ in range(5):
        Xt = c.get_particles()
        a_ref, _ = oracle.median_scale(Xt)
        G = oracle.logp_grad_gmm(Xt, mus, covs)
        ph_ref = oracle.phi(Xt, G, a_ref)
        c.step_with_model(model)
        a_dev, _, _ = c.last_scale()
        assert a_dev == pytest.approx(a_ref, rel=1e-12)
        Xref = Xt.copy()
        oracle.apply_update(Xref, o_opt.step(ph_ref), lo, up)
        Xdev = c.get_particles()
        # increments are lr * O(1) -> compare positions with the phi tolerance
        assert np.max(np.abs(Xdev - Xref)) <= 1e-9


def test_optimizer_bit_exact(oracle):
    """Same phi in -> bit-identical optimizer increments and clamp."""
    n, d = 100, 3
    X = oracle.splitmix((n, d), 1.0, 7)
    G = oracle.splitmix((n, d), 1.0, 8)
    c = _ctx(X)
    c.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999, 1e-8)
    c.set_scale(C.SVGD_SCALE_FIXED, 0.5)
    c.set_bounds(np.full(d, -0.9), np.full(d, 0.9))
    o_opt = oracle.Adam((n, d), 0.1, 0.9, 0.999)
    Xo = X.copy()
    for _ in range(3):
        ph = c.phi(G, 0.5)  # the device's own phi for this X
        c.check(c.lib.svgd_step(c.h, C.dptr(np.ascontiguousarray(G))))
        oracle.apply_update(Xo, o_opt.step(ph), np.full(d, -0.9), np.full(d, 0.9))
        np.testing.assert_array_equal(c.get_particles(), Xo)


def test_api_errors():
    with pytest.raises(ValueError, match=r"SVGDCpp: \[Argument Error\] Invalid value for decay"):
        S.Adam(2, 10, 0.1, 1.0, 0.9)
    X = np.zeros((2, 10))
    k = S.GaussianRBFKernel(X)
    m = S.MultivariateNormal([0.0, 0.0], np.eye(2))
    with pytest.raises(S.DimensionMismatchException, match=r"SVGDCpp: \[Dimension Error\]"):
        S.SVGD(3, 10, X, k, m, S.Adam(2, 10, 0.1, 0.9, 0.999))
    with pytest.raises(ValueError, match="Invalid Model object pointer"):
        S.SVGD(2, 10, X, k, None, S.Adam(2, 10, 0.1, 0.9, 0.999))
    c = S.Context(2, 10)
    with pytest.raises(S.UnsetException):
        c.median_scale()  # particles unset
    rc = c.lib.svgd_set_optimizer(c.h, C.SVGD_OPT_ADAM, 0.1, 1.5, 0.9, 1e-8)
    assert rc == C.SVGD_ERR_ARG and b"decay parameter beta" in c.lib.svgd_last_error(c.h)


def test_svgd_class_matches_manual_loop(oracle):
    """test_svgd.cpp structure: the SVGD class vs a manual loop on the same
    device primitives (median, phi, optimizer) -- here the manual loop is the
    oracle, the class is the Python mirror over the C ABI."""
    n, d = 50, 2
    X0 = oracle.eigen_random(d, n, 3.0, 1)
    mvn = S.MultivariateNormal([-0.6871, 0.8010], 5 * np.array([[0.2260, 0.1652], [0.1652, 0.6779]]))
    coord = np.ascontiguousarray(X0.T)  # (d, n) like Eigen
    kern = S.GaussianRBFKernel(coord, S.GaussianRBFKernel.ScaleMethod.Median, mvn)
    opt = S.Adam(d, n, 0.1, 0.9, 0.999)
    svgd = S.SVGD(d, 30, coord, kern, mvn, opt)
    svgd.Initialize()
    svgd.Run()
    Xo = oracle.run_svgd(X0, lambda X: oracle.logp_grad_gmm(X, np.array([[-0.6871, 0.8010]]),
                                                            5 * np.array([[[0.2260, 0.1652], [0.1652, 0.6779]]])),
                         30, oracle.Adam((n, d), 0.1, 0.9, 0.999))
    np.testing.assert_allclose(coord.T, Xo, rtol=0, atol=1e-8)
