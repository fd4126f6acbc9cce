"""Bracket tracking (speculative steps): the collect pass's bracket predicted
from the previous steps' selected medians instead of a sample.  GPU only.

The median stays an exact order statistic of all N^2 distances
(GaussianRBFKernel.hpp:164-188) whatever the bracket, so a tracked run must be
BIT-IDENTICAL to one that samples every bracket (SVGD_TRACK_BRACKET=0), also
when every predicted bracket misses (a failed plan: the step is restored and
redone with a sampled bracket).
"""
import numpy as np
import pytest

import svgdcpp_amd as S
from svgdcpp_amd import _capi as C

pytestmark = pytest.mark.gpu


def _pair(oracle, monkeypatch, n, d, env, dtype=None):
    X = oracle.splitmix((n, d), 3.0, 11 * n + d)
    mus = oracle.splitmix((3, d), 2.0, 17)
    model = S.GaussianSum(list(mus), [np.eye(d) * (1.0 + 0.25 * k) for k in range(3)])
    ctxs = []
    for tr in ("1", "0"):
        monkeypatch.setenv("SVGD_TRACK_BRACKET", tr)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        c = S.Context(d, n) if dtype is None else S.Context(d, n, dtype=dtype)
        c.set_particles(X)
        c.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999, 1e-8)
        ctxs.append(c)
    return ctxs, model


@pytest.mark.parametrize("n,d,dtype", [(6000, 8, None), (9000, 2, None), (7000, 5, None),
                                       (6000, 24, None), (6000, 64, "f32")])
def test_tracked_brackets_bit_identical(oracle, monkeypatch, n, d, dtype):
    """Row path (d <= 16), fp64 tile path (d = 24) and the F32 tile path."""
    dt = None if dtype is None else C.SVGD_F32
    (a, b), model = _pair(oracle, monkeypatch, n, d, {}, dt)
    a.diagnostics()
    for step in range(16):
        for c in (a, b):
            c.step_with_model(model)
        assert np.array_equal(a.get_particles(), b.get_particles()), step
        assert a.last_scale()[:2] == b.last_scale()[:2], step
    da, db = a.diagnostics(), b.diagnostics()
    # predicted once the prediction errors are small enough for a bracket
    # narrower than the sampled one (quadratic extrapolation needs 3 medians;
    # the d = 24 / 64 trajectories settle later)
    assert da["trk_steps"] >= (3 if d <= 16 else 1)
    assert db["trk_steps"] == 0
    a.close()
    b.close()


def test_tracked_misses_are_redone(oracle, monkeypatch):
    """A half-width far below the median's step-to-step motion: every
    predicted bracket misses, each such step is redone with a sampled bracket,
    and the trajectory is unchanged."""
    env = {"SVGD_TRACK_ERR_MULT": "0", "SVGD_TRACK_MIN_WIDTH": "1e-14"}
    (a, b), model = _pair(oracle, monkeypatch, 6000, 8, env)
    a.diagnostics()
    for step in range(10):
        for c in (a, b):
            c.step_with_model(model)
        assert np.array_equal(a.get_particles(), b.get_particles()), step
    da = a.diagnostics()
    assert da["trk_steps"] >= 3
    assert da["trk_miss"] == da["trk_steps"]
    a.close()
    b.close()
