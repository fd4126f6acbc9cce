"""Every BASELINE.json configuration at its full size on one GPU.  GPU only.

The oracle cannot hold n^2 distances at these sizes, so parity is checked
through size-independent properties:

  * median selection: the bracket path (the default at these sizes) and the
    forced streamed radix fallback (candidate capacity 1: every region
    overflows) select BIT-IDENTICAL order statistics -- two independent
    algorithms over all n(n-1)/2 keys (GaussianRBFKernel.hpp:164-188,222-254);
  * the selected squared distances have the right ranks among ALL pairs,
    counted on the CPU in one streamed pass of the direct form (64-bit counts:
    N = 262144 has 3.4e10 pairs, past 2^32):  count(D^2 < s(1-eps)) <= rank <
    count(D^2 < s(1+eps)), eps = 1e-12 (fp64; the centred Gram form differs in
    the last bits) or 1e-5 (fp32 keys);
  * phi_hat on 1024 sampled rows (the first and last 256, 512 around n / 2) vs the oracle's phi
    for those rows against all N columns (SVGD.hpp:407-454): max-abs <= 1e-10
    (fp64) or <= 1e-4 max|phi_hat| (fp32, cfg5);
  * one full step (scale + host grad log p + phi_hat + Adam) on the sampled
    rows vs the oracle's Adam update from the device's scale: <= 1e-9 (fp64).

Configurations (BASELINE.json configs[1..4], bench.py CONFIGS): cfg2 N=16384
d=2 MVN (the d = 2 bracket path at full size), cfg3 N=65536 d=8 GMM(k=4),
cfg4's N=262144 d=8 on one GPU (no 32-bit count/index overflow), cfg5
N=65536 d=64 fp32.
"""
import numpy as np
import pytest

import bench
import svgdcpp_amd as S
from svgdcpp_amd import _capi as C

pytestmark = pytest.mark.gpu

CASES = [
    ("cfg2", 16384, 2, C.SVGD_F64),
    ("cfg3", 65536, 8, C.SVGD_F64),
    ("cfg4", 262144, 8, C.SVGD_F64),
    ("cfg5", 65536, 64, C.SVGD_F32),
]


def _workload(name, n, d):
    X0, mus, covs = bench.config_workload(name, n, d, 4)
    return X0, S.GaussianSum(list(mus), list(covs))


def _ctx(X, dtype):
    n, d = X.shape
    c = S.Context(d, n, dtype=dtype)
    c.set_particles(X)
    return c


def _sample_rows(n):
    # both ends and 512 mid-range rows straddling n / 2: a k_phi_rows row
    # block boundary (1024 rows at d = 8), a symmetric-pass block boundary
    # and, on one rank, the middle of the column-split range
    return [(0, 256), (n // 2 - 256, n // 2 + 256), (n - 256, n)]


@pytest.mark.parametrize("name,n,d,dtype", CASES, ids=[c[0] for c in CASES])
def test_fullsize_median_bracket_equals_fallback_and_ranks(oracle, name, n, d, dtype):
    X, _ = _workload(name, n, d)
    c = _ctx(X, dtype)
    a, med = c.median_scale()
    path = c.last_scale()[2]
    assert path in (C.SVGD_MEDIAN_BRACKET, C.SVGD_MEDIAN_REBRACKET)
    s_lo, s_hi, r_lo, r_hi = c.last_median_keys()
    c.close()
    # forced fallback: streamed radix select over every pair
    f = _ctx(X, dtype)
    f.set_median_tuning(candidate_capacity=1)
    af, medf = f.median_scale()
    assert f.last_scale()[2] == C.SVGD_MEDIAN_FALLBACK
    fk = f.last_median_keys()
    f.close()
    assert (af, medf) == (a, med)
    assert fk == (s_lo, s_hi, r_lo, r_hi)
    assert med == (np.sqrt(s_lo) + np.sqrt(s_hi)) / 2 and a == np.log(n) / (med * med)
    # ranks among all n(n-1)/2 direct-form distances (64-bit CPU counts)
    eps = 1e-5 if dtype == C.SVGD_F32 else 1e-12
    assert 0 <= r_lo <= r_hi and 0 < s_lo <= s_hi
    cnt = oracle.upper_sqdist_counts(X, [s_lo * (1 - eps), s_lo * (1 + eps), s_hi * (1 - eps), s_hi * (1 + eps)])
    assert cnt[0] <= r_lo < cnt[1], (s_lo, r_lo, cnt)
    assert cnt[2] <= r_hi < cnt[3], (s_hi, r_hi, cnt)


@pytest.mark.parametrize("name,n,d,dtype", CASES, ids=[c[0] for c in CASES])
def test_fullsize_phi_rows_match_oracle(oracle, name, n, d, dtype):
    X, model = _workload(name, n, d)
    G = model.log_model_grad(X)
    c = _ctx(X, dtype)
    a, _ = c.median_scale()
    ph = c.phi(G, a)
    c.close()
    assert np.all(np.isfinite(ph))
    for r0, r1 in _sample_rows(n):
        ref = oracle.phi(X, G, a, rows=(r0, r1))
        err = np.max(np.abs(ph[r0:r1] - ref))
        if dtype == C.SVGD_F32:
            assert err <= 1e-4 * np.max(np.abs(ref)), err
        else:
            assert err <= 1e-10, err


@pytest.mark.parametrize("name,n,d,dtype", [c for c in CASES if c[3] == C.SVGD_F64],
                         ids=[c[0] for c in CASES if c[3] == C.SVGD_F64])
def test_fullsize_step_rows_match_oracle(oracle, name, n, d, dtype):
    X, model = _workload(name, n, d)
    c = _ctx(X, dtype)
    c.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999, 1e-8)
    c.step_with_model(model)
    a = c.last_scale()[0]
    X1 = c.get_particles()
    c.close()
    G = model.log_model_grad(X)
    for r0, r1 in _sample_rows(n):
        ph = oracle.phi(X, G, a, rows=(r0, r1))
        Xr = X[r0:r1].copy()
        oracle.apply_update(Xr, oracle.Adam((r1 - r0, d), 0.1, 0.9, 0.999).step(ph))
        assert np.max(np.abs(X1[r0:r1] - Xr)) <= 1e-9


def test_fullsize_rebracket_path_exact(monkeypatch):
    """cfg3 with a zero-width sample bracket: the re-bracket (wider bracket,
    second collect pass) selects the same keys as the normal bracket."""
    X, _ = _workload("cfg3", 65536, 8)
    c = _ctx(X, C.SVGD_F64)
    ref = c.median_scale()
    c.close()
    monkeypatch.setenv("SVGD_MEDIAN_SIGMA", "0")
    r = _ctx(X, C.SVGD_F64)
    got = r.median_scale()
    path = r.last_scale()[2]
    r.close()
    assert got == ref
    assert path in (C.SVGD_MEDIAN_BRACKET, C.SVGD_MEDIAN_REBRACKET)


def test_fullsize_plain_form_with_outlier(oracle):
    """cfg3 plus one far outlier: a log2e max|xc|^2 >> 300, so every wave of
    the phi row stream takes the plain (unfolded, clamped-exponent) form and
    the symmetric pass hands the step over -- sampled rows, the outlier's own
    row included, against the oracle."""
    X, model = _workload("cfg3", 65536, 8)
    X = X.copy()
    X[70] += 60.0
    G = model.log_model_grad(X)
    c = _ctx(X, C.SVGD_F64)
    a, _ = c.median_scale()
    ph = c.phi(G, a)
    c.close()
    assert np.all(np.isfinite(ph))
    for r0, r1 in [(0, 256)] + _sample_rows(65536)[1:]:
        ref = oracle.phi(X, G, a, rows=(r0, r1))
        assert np.max(np.abs(ph[r0:r1] - ref)) <= 1e-10, (r0, r1)


def test_fullsize_five_speculative_steps(oracle):
    """cfg3, 5 steps: queued back to back (speculative device plan, no host
    round trip inside a step) they end bit-identical to 5 steps run one at a
    time, and every one of those steps matches the oracle's step on the
    sampled rows from the device's scale of that X_t (<= 1e-9)."""
    X0, model = _workload("cfg3", 65536, 8)
    b2b = _ctx(X0, C.SVGD_F64)
    b2b.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999, 1e-8)
    for _ in range(5):
        b2b.step_with_model(model)
    X5 = b2b.get_particles()
    b2b.close()
    c = _ctx(X0, C.SVGD_F64)
    c.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999, 1e-8)
    rows = _sample_rows(65536)
    opts = {r: oracle.Adam((r[1] - r[0], 8), 0.1, 0.9, 0.999) for r in rows}
    Xt = X0
    for _ in range(5):
        c.step_with_model(model)
        a = c.last_scale()[0]
        X1 = c.get_particles()
        G = model.log_model_grad(Xt)
        for r0, r1 in rows:
            ph = oracle.phi(Xt, G, a, rows=(r0, r1))
            Xr = Xt[r0:r1].copy()
            oracle.apply_update(Xr, opts[(r0, r1)].step(ph))
            assert np.max(np.abs(X1[r0:r1] - Xr)) <= 1e-9
        Xt = X1
    c.close()
    assert np.array_equal(Xt, X5)
