"""The speculative step (device-side bucket plan, no mid-step host round trip).
GPU only.

After a step whose median took the bucket path, the next step plans the
bucket select on the device and the host checks the plan's status only before
the next call that depends on the step.  A failed plan (bracket miss,
overflowed region, oversized buckets) restores X_t, m_t, v_t, t and redoes the
step on the synchronous path.  Either way the trajectory must be BIT-IDENTICAL
to the synchronous path (SVGD_SPECULATE=0): the median is exact on every path
(GaussianRBFKernel.hpp:164-188, SVGD.hpp:373-400).
"""
import numpy as np
import pytest

import svgdcpp_amd as S
from svgdcpp_amd import _capi as C

pytestmark = pytest.mark.gpu


def _ctx(monkeypatch, X, spec):
    monkeypatch.setenv("SVGD_SPECULATE", "1" if spec else "0")
    n, d = X.shape
    c = S.Context(d, n)
    c.set_particles(X)
    c.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999, 1e-8)
    return c


@pytest.mark.parametrize("n,d", [(6000, 8), (9000, 2), (7000, 13)])
def test_speculative_steps_bit_identical(oracle, monkeypatch, n, d):
    X = oracle.splitmix((n, d), 3.0, n + d)
    mus = oracle.splitmix((3, d), 2.0, 7)
    model = S.GaussianSum(list(mus), [np.eye(d) * (1.0 + 0.25 * k) for k in range(3)])
    a = _ctx(monkeypatch, X, True)
    b = _ctx(monkeypatch, X, False)
    paths = []
    # 4 normal steps, 2 with a 1-key candidate capacity (every region overflows:
    # the speculative plan fails and the step is redone on the exact streamed
    # fallback), then 3 normal steps again
    for step in range(9):
        cap = 1 if step in (4, 5) else 0
        for c in (a, b):
            c.set_median_tuning(candidate_capacity=cap)
            c.step_with_model(model)
        xa, xb = a.get_particles(), b.get_particles()
        assert np.array_equal(xa, xb), step
        sa, sb = a.last_scale(), b.last_scale()
        assert sa[:2] == sb[:2], step
        paths.append(sa[2])
    assert C.SVGD_MEDIAN_FALLBACK in paths
    a.close()
    b.close()


def test_speculative_matches_oracle_trajectory(oracle, monkeypatch):
    """Five speculative steps against the oracle's SVGD::Step (phi, Adam)."""
    n, d = 6000, 8
    X = oracle.splitmix((n, d), 3.0, 5)
    mus = oracle.splitmix((4, d), 3.0, 6)
    covs = np.stack([np.eye(d) * (1.0 + 0.25 * k) for k in range(4)])
    model = S.GaussianSum(list(mus), list(covs))
    c = _ctx(monkeypatch, X, True)
    opt = oracle.Adam((n, d), 0.1, 0.9, 0.999)
    Xr = X.copy()
    for _ in range(5):
        a_ref, _ = oracle.median_scale(Xr)
        G = oracle.logp_grad_gmm(Xr, mus, covs)
        c.step_with_model(model)
        a_dev = c.last_scale()[0]
        assert a_dev == pytest.approx(a_ref, rel=1e-12)
        ph = oracle.phi(Xr, G, a_dev)
        oracle.apply_update(Xr, opt.step(ph))
        assert np.max(np.abs(c.get_particles() - Xr)) <= 1e-9
    c.close()
