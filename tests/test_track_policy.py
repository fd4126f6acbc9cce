"""The premise of the tracked median bracket (svgd_capi.cpp trk_predict):
along an SVGD trajectory the median of D^2 moves smoothly enough that a
quadratic extrapolation of the last three selected medians, with a half-width
of 4x the largest of the last three prediction errors, contains the next
median.  CPU only: the oracle's own trajectory (GaussianRBFKernel.hpp:164-188
median, SVGD.hpp:373-400 step, Adam), the policy restated in Python."""
import numpy as np
import pytest


def _policy(m, mult=4.0, wmin=2e-5):
    hist, errs, used, miss, ws = [], [], 0, 0, []
    for mt in m:
        if len(hist) >= 2:
            p = 3 * hist[-1] - 3 * hist[-2] + hist[-3] if len(hist) >= 3 else 2 * hist[-1] - hist[-2]
            if p <= 0:
                p = hist[-1]
            e = max(errs[-3:]) if errs else abs(hist[-1] - hist[-2]) / hist[-1]
            w = max(mult * e, wmin)
            err = abs(mt - p) / mt
            errs.append(err)
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
