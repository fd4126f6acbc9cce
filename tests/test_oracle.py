"""Pin the CPU oracle against the reference's own published outputs and
known-answer cases.  CPU only."""
import json
import os

import numpy as np
import pytest


def _load(golden_dir, name):
    with open(os.path.join(golden_dir, name)) as f:
        return json.load(f)


def _optimizer(o, spec, shape):
    if spec["kind"] == "adam":
        return o.Adam(shape, spec["lr"], spec["beta1"], spec["beta2"])
    if spec["kind"] == "adagrad":
        return o.AdaGrad(shape, spec["lr"])
    return o.RMSProp(shape, spec["lr"], spec["beta"])


@pytest.mark.parametrize("case", ["mvn", "gmm"])
def test_oracle_reproduces_published_notebook(oracle, golden_dir, case):
    """examples/*/ *.ipynb final particle tables, 1000 iterations, 6 digits."""
    nb = _load(golden_dir, "notebooks.json")[case]
    n, d = nb["n"], nb["d"]
    X0 = oracle.eigen_random(d, n, nb["init_scale"], nb["seed"])
    # initial coordinates printed by the notebook (6 significant digits)
    np.testing.assert_allclose(X0, np.array(nb["initial"]), rtol=5e-6, atol=1e-6)
    mus, covs = np.array(nb["means"]), np.array(nb["covs"])
    X = oracle.run_svgd(X0, lambda X: oracle.logp_grad_gmm(X, mus, covs), nb["iters"],
                        _optimizer(oracle, nb["optimizer"], (n, d)))
    np.testing.assert_allclose(X, np.array(nb["final"]), rtol=5e-6, atol=1e-6)


def test_oracle_test_svgd_scenario(oracle, golden_dir):
    """tests/test_svgd.cpp scenario: fixed kernel exp(-|x-x'|^2), Adam, bounds."""
    from golden.make_golden import test_svgd_model_grad  # noqa: E402
    g = _load(golden_dir, "test_svgd_n10.json")
    X0 = oracle.eigen_random(2, 10, 1.0, 1)
    np.testing.assert_array_equal(X0, np.array(g["initial"]))
    X = oracle.run_svgd(X0, test_svgd_model_grad, g["iters"], oracle.Adam((10, 2), 0.1, 0.9, 0.999),
                        scale=1.0, lower=np.array(g["lower"]), upper=np.array(g["upper"]))
    np.testing.assert_array_equal(X, np.array(g["final"]))
    # the values the survey quotes for this scenario
    np.testing.assert_allclose(X[:, 0][:4], [1, 1, 0.3111949417, -0.4702737921], atol=1e-10)
    np.testing.assert_allclose(X[:, 1][:4], [-0.2702913453, 0.5551141973, -1, 0.836541188], atol=1e-10)


def _median_numpy(X):
    """Straight numpy restatement of GaussianRBFKernel::ComputeScale (Median)."""
    S = X @ X.T
    dg = np.diag(S)
    D2 = (dg[:, None] + dg[None, :]) - 2 * S
    np.fill_diagonal(D2, 0.0)
    dist = np.sqrt(np.maximum(D2, 0)).reshape(-1)
    v = np.sort(dist)
    c = v.size
    med = (v[c // 2 - 1] + v[c // 2]) / 2 if c % 2 == 0 else v[c // 2]
    return np.log(X.shape[0]) / med ** 2, med


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8, 9, 31, 64, 65, 200])
@pytest.mark.parametrize("d", [1, 2, 5])
def test_oracle_median_edge_cases(oracle, n, d):
    X = oracle.splitmix((n, d), 2.0, 1000 + n * 7 + d)
    a, med = oracle.median_scale(X)
    a2, med2 = _median_numpy(X)
    assert med == pytest.approx(med2, rel=1e-13)
    assert a == pytest.approx(a2, rel=1e-12)


def test_oracle_median_upper_triangle_identity(oracle):
    """The device selects on upper-triangle squared distances; check the rank
    mapping (plan) against the full n^2 list for odd and even n."""
    for n in range(2, 40):
        X = oracle.splitmix((n, 3), 1.0, 77 + n)
        full = np.sqrt(np.maximum(((X[:, None, :] - X[None, :, :]) ** 2).sum(-1), 0)).reshape(-1)
        v = np.sort(full)
        c = v.size
        ref = (v[c // 2 - 1] + v[c // 2]) / 2 if c % 2 == 0 else v[c // 2]
        iu = np.triu_indices(n, 1)
        u = np.sort(((X[iu[0]] - X[iu[1]]) ** 2).sum(-1))

        def at(k):
            return 0.0 if k < n else np.sqrt(u[(k - n) // 2])
        got = (at(c // 2 - 1) + at(c // 2)) / 2 if c % 2 == 0 else at(c // 2)
        assert got == pytest.approx(ref, rel=1e-14)


def test_oracle_phi_matches_definition(oracle):
    """phi_hat = (1/N)(G K + [I..I] Kg) -- numpy restatement of SVGD.hpp:453."""
    n, d = 40, 3
    X = oracle.splitmix((n, d), 1.5, 5)
    G = oracle.splitmix((n, d), 1.0, 6)
    a = 0.7
    ph, K, Kg = oracle.phi(X, G, a, materialise=True)
    diff = X[None, :, :] - X[:, None, :]  # [i, j] = x_j - x_i
    Kr = np.exp(-a * (diff ** 2).sum(-1))
    Kgr = -2 * a * diff * Kr[..., None]
    np.testing.assert_allclose(K, Kr, rtol=1e-14)
    np.testing.assert_allclose(Kg, Kgr, rtol=1e-13, atol=1e-15)
    ref = (Kr @ G + Kgr.sum(1)) / n
    np.testing.assert_allclose(ph, ref, rtol=1e-12, atol=1e-14)
    # row-sharded evaluation is the same computation
    np.testing.assert_array_equal(oracle.phi(X, G, a, rows=(10, 25)), ph[10:25])


def test_oracle_optimizers_match_reference_formulas(oracle):
    rng = np.random.default_rng(0)
    g1, g2 = rng.normal(size=(7, 3)), rng.normal(size=(7, 3))
    ad = oracle.Adam((7, 3), 0.1, 0.9, 0.999)
    d1, d2 = ad.step(g1), ad.step(g2)
    m = 0.9 * (0.1 * g1) + 0.1 * g2
    v = 0.999 * (0.001 * g1 * g1) + 0.001 * g2 * g2
    ref = 0.1 * (1 / (1e-8 + np.sqrt(v / (1 - 0.999 ** 2)))) * (m / (1 - 0.9 ** 2))
    np.testing.assert_allclose(d2, ref, rtol=1e-13)
    ag = oracle.AdaGrad((7, 3), 0.1)
    ag.step(g1)
    np.testing.assert_allclose(ag.step(g2), 0.1 / (1e-8 + np.sqrt(g1 ** 2 + g2 ** 2)) * g2, rtol=1e-13)
    rp = oracle.RMSProp((7, 3), 0.01, 0.9)
    rp.step(g1)
    vv = 0.9 * (0.1 * g1 ** 2) + 0.1 * g2 ** 2
    np.testing.assert_allclose(rp.step(g2), 0.01 / (1e-8 + np.sqrt(vv)) * g2, rtol=1e-13)
    with pytest.raises(ValueError, match="SVGDCpp: "):
        oracle.Adam((1, 1), 0.1, 1.0, 0.5)
    with pytest.raises(ValueError, match="SVGDCpp: "):
        oracle.RMSProp((1, 1), 0.1, 1.5)


def test_oracle_clamp_order(oracle):
    """SVGD.hpp:398: min(upper) then max(lower) (lower wins if bounds cross)."""
    X = np.array([[0.5, 3.0], [-2.0, 0.0]])
    oracle.apply_update(X, np.zeros_like(X), lower=np.array([1.0, -1.0]), upper=np.array([0.0, 1.0]))
    np.testing.assert_array_equal(X, [[1.0, 1.0], [1.0, 0.0]])


def test_golden_phi_fixtures_consistent(oracle, golden_dir):
    for name in ["n256_d2", "n77_d3"]:
        z = np.load(os.path.join(golden_dir, f"phi_{name}.npz"))
        a, med = oracle.median_scale(z["X"])
        assert a == z["a"] and med == z["med"]
        np.testing.assert_array_equal(oracle.phi(z["X"], z["G"], a), z["phi"])


def test_hessian_sum_matches_finite_differences(oracle):
    """oracle.neg_hess_sum_gmm (the Hessian scale's sum, GaussianRBFKernel.hpp:
    197-205) against central differences of the oracle's own gradient."""
    rng = np.random.default_rng(0)
    d, n = 3, 40
    X = rng.standard_normal((n, d))
    mus = rng.standard_normal((2, d))
    covs = np.stack([np.eye(d) * 1.5, np.eye(d) * 0.7 + 0.1])
    H = oracle.neg_hess_sum_gmm(X, mus, covs)
    Hfd = np.zeros((d, d))
    h = 1e-5
    for i in range(n):
        for l in range(d):
            e = np.zeros(d)
            e[l] = h
            gp = oracle.logp_grad_gmm((X[i] + e)[None], mus, covs)[0]
            gm = oracle.logp_grad_gmm((X[i] - e)[None], mus, covs)[0]
            Hfd[:, l] -= (gp - gm) / (2 * h)
    assert np.max(np.abs(H - Hfd)) < 1e-7
    np.testing.assert_array_equal(H, H.T)


def test_phi_matrix_reduces_to_isotropic(oracle):
    rng = np.random.default_rng(1)
    X = rng.standard_normal((60, 4))
    G = rng.standard_normal((60, 4))
    a = 0.37
    np.testing.assert_allclose(oracle.phi_matrix(X, G, a * np.eye(4)), oracle.phi(X, G, a),
                               rtol=1e-13, atol=1e-15)
