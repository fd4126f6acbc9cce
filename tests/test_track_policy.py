"""The premise of the tracked median bracket (svgd_capi.cpp trk_predict):
along an SVGD trajectory the median of D^2 moves smoothly enough that an
extrapolation of the last selected medians -- the quadratic one (3 points,
half-width mult x the largest of its last three relative errors) or the cubic
one (4 points, half-width 2 mult x its own), whichever half-width is narrower
-- contains the next median.  CPU only: the oracle's own trajectory
(GaussianRBFKernel.hpp:164-188 median, SVGD.hpp:373-400 step, Adam), the
policy restated in Python."""
import numpy as np
import pytest


def _extrap(h, order):
    if order == 3 and len(h) >= 4:
        p = 4 * h[-1] - 6 * h[-2] + 4 * h[-3] - h[-4]
    elif len(h) >= 3:
        p = 3 * h[-1] - 3 * h[-2] + h[-3]
    else:
        p = 2 * h[-1] - h[-2]
    return p if p > 0 else h[-1]


def _policy(m, mult=4.0, wmin=2e-5):
    hist, eq, ec, used, miss, ws, cubic = [], [], [], 0, 0, [], 0
    for mt in m:
        if len(hist) >= 2:
            pq = _extrap(hist, 2)
            pc = _extrap(hist, 3) if len(hist) >= 4 else None
            e = max(eq[-3:]) if eq else abs(hist[-1] - hist[-2]) / hist[-1]
            w, p = mult * e, pq
            if pc is not None and len(ec) >= 3 and 2 * mult * max(ec[-3:]) < w:
                w, p = 2 * mult * max(ec[-3:]), pc
                cubic += 1
            w = max(w, wmin)
            err = abs(mt - p) / mt
            eq.append(abs(mt - pq) / mt)
            if pc is not None:
                ec.append(abs(mt - pc) / mt)
            if w < 0.05:
                used += 1
                ws.append(w)
                miss += err > w
        hist.append(mt)
    return used, miss, ws


# (the median of a small N has more step-to-step jitter: at N = 2048, d = 8
# one of 37 predictions misses -- a redo, not an error; none at these sizes)
@pytest.mark.parametrize("n,d", [(4096, 8), (3000, 2)])
def test_tracked_bracket_policy_on_oracle_trajectory(oracle, n, d):
    X = oracle.splitmix((n, d), 3.0, 0x5EED)
    mus = oracle.splitmix((4, d), 3.0, 0x5EEE)
    covs = np.stack([np.eye(d) * (1.0 + 0.25 * q) for q in range(4)])
    opt = oracle.Adam((n, d), 0.1, 0.9, 0.999)
    meds = []
    for _ in range(40):
        a, med = oracle.median_scale(X)
        meds.append(med * med)
        G = oracle.logp_grad_gmm(X, mus, covs)
        oracle.apply_update(X, opt.step(oracle.phi(X, G, a)))
    used, miss, ws = _policy(np.array(meds))
    assert used >= 35
    assert miss == 0
    # narrow: the median half-width well under 1 % of the median
    assert np.median(ws) < 5e-3
