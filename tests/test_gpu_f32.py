"""fp32 compute path (SVGD_F32) against the fp64 oracle.  GPU only.

The O(N^2) work (median distances, kernel values, phi contraction) runs on the
fp32 MFMA tile kernels; centring, the phi epilogue and the optimizer stay fp64.

Tolerances (written here):
  * phi_hat vs the fp64 oracle from identical (X, G, a):  max-abs <= 1e-4 * max|phi_hat|
  * median / scale a vs the fp64 oracle:                rel <= 1e-5
  * median selection:  BIT-EXACT order statistics of the device's own fp32 keys
    (svgd_debug_pair_keys), on the direct, bracket and fallback paths
"""
import numpy as np
import pytest

import svgdcpp_amd as S
from svgdcpp_amd import _capi as C

pytestmark = pytest.mark.gpu

REL = 1e-4


def _ctx(X):
    n, d = X.shape
    c = S.Context(d, n, dtype=C.SVGD_F32)
    c.set_particles(X)
    return c


@pytest.mark.parametrize("n,d", [(300, 64), (1000, 64), (2000, 33), (777, 8), (500, 2), (129, 17)])
def test_f32_phi_matches_oracle(oracle, n, d):
    X = oracle.splitmix((n, d), 3.0, 500 + n + d)
    G = oracle.splitmix((n, d), 1.0, 600 + n + d)
    a = float(np.log(n) / (2.0 * d * 3.0))  # typical median-heuristic magnitude
    ph = _ctx(X).phi(G, a)
    ref = oracle.phi(X, G, a)
    assert np.all(np.isfinite(ph))
    assert np.max(np.abs(ph - ref)) <= REL * np.max(np.abs(ref))


@pytest.mark.parametrize("n,d", [(400, 64), (333, 5)])
def test_f32_median_exact_on_own_keys(oracle, n, d):
    X = oracle.splitmix((n, d), 2.0, 7 * n + d)
    c = _ctx(X)
    a, med = c.median_scale()
    keys = np.empty(n * (n - 1) // 2)
    c.check(c.lib.svgd_debug_pair_keys(c.h, C.dptr(keys), keys.size))
    # every key is an fp32 value (widened exactly)
    assert np.array_equal(keys.astype(np.float32).astype(np.float64), keys)
    iu = np.triu_indices(n, 1)
    ref_keys = ((X[iu[0]] - X[iu[1]]) ** 2).sum(-1)
    np.testing.assert_allclose(keys, ref_keys, rtol=1e-4, atol=1e-4)
    u = np.sort(keys)
    tot = n * n

    def at(k):
        return 0.0 if k < n else np.sqrt(u[(k - n) // 2])
    exp = (at(tot // 2 - 1) + at(tot // 2)) / 2 if tot % 2 == 0 else at(tot // 2)
    assert med == exp
    assert med == pytest.approx(oracle.median_scale(X)[1], rel=1e-5)
    assert a == pytest.approx(np.log(n) / (exp * exp), rel=1e-15)


def test_f32_median_bracket_and_fallback_agree(oracle):
    n, d = 1500, 24
    X = oracle.splitmix((n, d), 1.0, 99)
    a0, m0 = _ctx(X).median_scale()  # direct
    c = _ctx(X)
    c.check(c.lib.svgd_set_median_tuning(c.h, 0, 1 << 14, -1))
    a1, m1 = c.median_scale()
    assert c.last_scale()[2] == C.SVGD_MEDIAN_BRACKET
    c2 = _ctx(X)
    c2.check(c2.lib.svgd_set_median_tuning(c2.h, 0, 1 << 12, 1))
    a2, m2 = c2.median_scale()
    assert c2.last_scale()[2] == C.SVGD_MEDIAN_FALLBACK
    assert m1 == m0 and m2 == m0 and a1 == a0 and a2 == a0


def test_f32_step_tracks_f64(oracle):
    """Per-step fp32 vs fp64 along one fp64 trajectory: at every step both
    contexts see the same X_t and G_t; the fp32 scale agrees to rel 1e-5 and
    the fp32 phi_hat (with the fp64 scale) is within REL * max|phi_hat| of the
    fp64 one.  (Positions after whole Adam steps are not compared: Adam's first
    increments are +-lr * sign(phi), so a phi component near 0 may flip sign.)"""
    n, d = 2048, 64
    X = oracle.splitmix((n, d), 3.0, 11)
    mu = oracle.splitmix((1, d), 0.5, 12)
    model = S.GaussianSum(mu, np.eye(d)[None])
    c64 = S.Context(d, n, dtype=C.SVGD_F64)
    c32 = S.Context(d, n, dtype=C.SVGD_F32)
    adam = oracle.Adam((n, d), 0.1, 0.9, 0.999)
    for _ in range(3):
        c64.set_particles(X)
        c32.set_particles(X)
        a64, _ = c64.median_scale()
        a32, _ = c32.median_scale()
        assert a32 == pytest.approx(a64, rel=1e-5)
        G = model.log_model_grad(X)
        ph64 = c64.phi(G, a64)
        ph32 = c32.phi(G, a64)
        assert np.all(np.isfinite(ph32))
        assert np.max(np.abs(ph32 - ph64)) <= REL * np.max(np.abs(ph64))
        X = X.copy()
        oracle.apply_update(X, adam.step(ph64))


def test_f32_matrix_scale(oracle):
    n, d = 600, 20
    X = oracle.splitmix((n, d), 2.0, 31)
    G = oracle.splitmix((n, d), 1.0, 32)
    B = oracle.splitmix((d, d), 0.2, 33)
    M = (B @ B.T + 0.5 * np.eye(d)) / d
    c = _ctx(X)
    c.set_scale_matrix(M)
    ph = c.phi(G, 0.0)
    ref = oracle.phi_matrix(X, G, M)
    assert np.max(np.abs(ph - ref)) <= REL * np.max(np.abs(ref))


@pytest.mark.parametrize("n,d", [(300, 13), (1000, 20), (2049, 33), (4096, 64), (777, 64)])
def test_streamed_tile_phi_matches_generic(oracle, monkeypatch, n, d):
    """k_phi_f32s (operand-ordered streamed columns) against the generic fp32
    tile kernel (SVGD_PHI_TILE_GENERIC=1) and the fp64 oracle."""
    X = oracle.splitmix((n, d), 2.0, n + 7 * d)
    G = oracle.splitmix((n, d), 1.0, n + d + 1)
    out = []
    for generic in (False, True):
        if generic:
            monkeypatch.setenv("SVGD_PHI_TILE_GENERIC", "1")
        c = S.Context(d, n, dtype=C.SVGD_F32)
        c.set_particles(X)
        a = 0.7 / d
        out.append(c.phi(G, a))
        c.close()
    ref = oracle.phi(X, G, a)
    scale = np.max(np.abs(ref))
    assert np.max(np.abs(out[0] - ref)) <= 1e-4 * scale
    assert np.max(np.abs(out[0] - out[1])) <= 1e-4 * scale


@pytest.mark.parametrize("n,d", [(300, 64), (1000, 64), (2049, 33), (4096, 64), (777, 32), (129, 17),
                                 (640, 40), (3001, 48)])
def test_b3_tile_phi_matches_oracle(oracle, monkeypatch, n, d):
    """k_phi_b3 (SVGD_PHI_B3=1: the F32 tile phi on the bf16 matrix cores,
    each fp32 operand as three bf16 parts and six part products per fp32
    product) against the fp64 oracle and the fp32-MFMA kernel k_phi_f32s, at
    the F32 tolerance; ragged N leaves a partial last row block and padded
    columns."""
    X = oracle.splitmix((n, d), 2.0, 3 * n + d)
    G = oracle.splitmix((n, d), 1.0, 3 * n + d + 1)
    a = 0.7 / d
    out = {}
    for v in ("1", "0"):
        monkeypatch.setenv("SVGD_PHI_B3", v)
        c = S.Context(d, n, dtype=C.SVGD_F32)
        c.set_particles(X)
        out[v] = c.phi(G, a)
        name = c.phi_kernel_name()
        c.close()
        assert name.startswith("k_phi_b3" if v == "1" else "k_phi_f32s"), name
    ref = oracle.phi(X, G, a)
    scale = np.max(np.abs(ref))
    assert np.all(np.isfinite(out["1"]))
    assert np.max(np.abs(out["1"] - ref)) <= REL * scale
    assert np.max(np.abs(out["1"] - out["0"])) <= REL * scale


@pytest.mark.parametrize("n,d", [(300, 64), (4096, 64), (2049, 33), (3001, 48), (777, 32)])
def test_b3_two_row_groups_bit_identical(oracle, monkeypatch, n, d):
    """k_phi_b3 with two 16-row groups per wave (SVGD_PHI_B3_RG=2; a measured
    wash against one at cfg5, profiles/r06_b3_rg_il_ab.txt) runs the same MFMAs into
    the same accumulators in the same order as one row group per wave: phi
    bit-identical, ragged N (a partial last row group) included; and within
    the F32 tolerance of the oracle."""
    X = oracle.splitmix((n, d), 2.0, 5 * n + d)
    G = oracle.splitmix((n, d), 1.0, 5 * n + d + 1)
    a = 0.7 / d
    out = {}
    for rg in ("1", "2"):
        monkeypatch.setenv("SVGD_PHI_B3_RG", rg)
        c = S.Context(d, n, dtype=C.SVGD_F32)
        c.set_particles(X)
        out[rg] = c.phi(G, a)
        name = c.phi_kernel_name()
        c.close()
        assert name.startswith("k_phi_b3") and name.endswith(", %s>" % rg), name
    assert np.array_equal(out["1"], out["2"])
    ref = oracle.phi(X, G, a)
    assert np.max(np.abs(out["2"] - ref)) <= REL * np.max(np.abs(ref))


def test_b3_matrix_scale_and_step(oracle, monkeypatch):
    """k_phi_b3 under a full-matrix scale (whitened coordinates) and inside
    the fused step (optimizer epilogue) against the fp64 oracle."""
    monkeypatch.setenv("SVGD_PHI_B3", "1")
    n, d = 600, 32
    X = oracle.splitmix((n, d), 2.0, 41)
    G = oracle.splitmix((n, d), 1.0, 42)
    B = oracle.splitmix((d, d), 0.2, 43)
    M = (B @ B.T + 0.5 * np.eye(d)) / d
    c = _ctx(X)
    c.set_scale_matrix(M)
    ph = c.phi(G, 0.0)
    ref = oracle.phi_matrix(X, G, M)
    assert np.max(np.abs(ph - ref)) <= REL * np.max(np.abs(ref))
    c.close()
    mu = oracle.splitmix((1, d), 0.5, 44)
    model = S.GaussianSum(mu, np.eye(d)[None])
    c32 = S.Context(d, n, dtype=C.SVGD_F32)
    c32.set_particles(X)
    c32.set_optimizer(C.SVGD_OPT_ADAM, 0.01, 0.9, 0.999, 1e-8)
    assert c32.phi_kernel_name().startswith("k_phi_b3")
    for _ in range(3):
        c32.step_with_model(model)
    assert np.all(np.isfinite(c32.get_particles()))
    c32.close()
