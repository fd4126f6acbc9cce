"""svgd_step_host_model: the X_t copy, the host gradient and the G upload
pipelined in row chunks (SVGD.hpp:373-400 with Model::EvaluateLogModelGrad,
Model.hpp:335-338).  GPU only.

The pipelined step must give the same trajectory, bit for bit, as the split
begin / gradient / finish calls (the same kernels on the same G), and match
the oracle's SVGD::Step.
"""
import numpy as np
import pytest

import svgdcpp_amd as S
from svgdcpp_amd import _capi as C

pytestmark = pytest.mark.gpu


def _ctx(X, dtype=C.SVGD_F64):
    n, d = X.shape
    c = S.Context(d, n, dtype=dtype)
    c.set_particles(X)
    c.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999, 1e-8)
    return c


@pytest.mark.parametrize("n,d,k,dtype", [(1500, 3, 2, C.SVGD_F64), (9000, 8, 4, C.SVGD_F64),
                                         (20000, 2, 1, C.SVGD_F64), (5000, 64, 1, C.SVGD_F32)])
def test_pipelined_step_matches_split_step(oracle, n, d, k, dtype):
    X = oracle.splitmix((n, d), 3.0, n + d + k)
    mus = oracle.splitmix((k, d), 2.0, 11)
    model = S.GaussianSum(list(mus), [np.eye(d) * (1.0 + 0.25 * c) for c in range(k)])
    a, b = _ctx(X, dtype), _ctx(X, dtype)
    for step in range(4):
        a.step_with_model(model, pipelined=True)
        b.step_with_model(model, pipelined=False)
        assert np.array_equal(a.get_particles(), b.get_particles()), step
        assert a.last_scale()[:2] == b.last_scale()[:2], step
    a.close()
    b.close()


def test_pipelined_step_matches_oracle(oracle):
    n, d = 6000, 8
    X = oracle.splitmix((n, d), 3.0, 21)
    mus = oracle.splitmix((4, d), 3.0, 22)
    covs = np.stack([np.eye(d) * (1.0 + 0.25 * c) for c in range(4)])
    model = S.GaussianSum(list(mus), list(covs))
    c = _ctx(X)
    opt = oracle.Adam((n, d), 0.1, 0.9, 0.999)
    Xr = X.copy()
    for _ in range(3):
        a_ref, _ = oracle.median_scale(Xr)
        G = oracle.logp_grad_gmm(Xr, mus, covs)
        c.step_with_model(model)
        a_dev = c.last_scale()[0]
        assert a_dev == pytest.approx(a_ref, rel=1e-12)
        oracle.apply_update(Xr, opt.step(oracle.phi(Xr, G, a_dev)))
        assert np.max(np.abs(c.get_particles() - Xr)) <= 1e-9
    c.close()


def test_pipelined_step_rejects_bad_model():
    X = np.zeros((100, 3))
    c = _ctx(X)
    other = S.GaussianSum([np.zeros(4)], [np.eye(4)])
    with pytest.raises(ValueError):
        c.step_with_model(other)
    c.close()


@pytest.mark.parametrize("n,d,k,frac", [(9000, 8, 4, "62"), (13001, 5, 2, "62"), (9000, 8, 4, "50"),
                                        (13001, 5, 2, "80")])
def test_row_halves_step_matches_oracle(oracle, monkeypatch, n, d, k, frac):
    """phi in two row parts (SVGD_PHI_SPLIT=1; by default a rank of several
    with > 2048 rows per gradient thread; the first part SVGD_PHI_SPLIT_FRAC
    percent of the rows): the first part's X_{t+1} goes to the host gradient
    while the second part's phi runs.  Each part sums its own column splits,
    so the trajectory matches the whole-rows one to fp64 rounding, and every
    step matches the oracle's."""
    monkeypatch.setenv("SVGD_PHI_SPLIT_FRAC", frac)
    X = oracle.splitmix((n, d), 3.0, 31 + d)
    mus = oracle.splitmix((k, d), 3.0, 32)
    covs = np.stack([np.eye(d) * (1.0 + 0.25 * c) for c in range(k)])
    model = S.GaussianSum(list(mus), list(covs))
    monkeypatch.setenv("SVGD_PHI_SPLIT", "1")
    a = _ctx(X)
    monkeypatch.setenv("SVGD_PHI_SPLIT", "0")
    b = _ctx(X)
    opt = oracle.Adam((n, d), 0.1, 0.9, 0.999)
    Xr = X.copy()
    for step in range(4):
        a_ref, _ = oracle.median_scale(Xr)
        G = oracle.logp_grad_gmm(Xr, mus, covs)
        a.step_with_model(model)
        b.step_with_model(model)
        a_dev = a.last_scale()[0]
        assert a_dev == pytest.approx(a_ref, rel=1e-12), step
        oracle.apply_update(Xr, opt.step(oracle.phi(Xr, G, a_dev)))
        Xa = a.get_particles()
        assert np.max(np.abs(Xa - Xr)) <= 1e-9, step
        assert np.max(np.abs(Xa - b.get_particles())) <= 1e-10, step
    a.diagnostics()
    a.close()
    b.close()


@pytest.mark.parametrize("n,d,k,split", [(3000, 8, 4, "0"), (9000, 3, 2, "1"), (700, 2, 1, "0"),
                                         (2000, 20, 1, "0")])
def test_host_mirror_bit_exact(oracle, monkeypatch, n, d, k, split):
    """Small shards (<= 1 MiB): the update epilogue stores X_{t+1} into the
    pinned host buffer the gradient reads (SVGD_X_MIRROR) instead of the
    copy-engine round trip.  Same kernels, same values: the trajectory is
    bit-identical to the copying path, row split included, and a
    set_particles in between invalidates the mirror (the diagnostics count
    the steps that read it)."""
    X = oracle.splitmix((n, d), 3.0, 40 + n + d)
    mus = oracle.splitmix((k, d), 2.0, 41)
    model = S.GaussianSum(list(mus), [np.eye(d) * (1.0 + 0.25 * c) for c in range(k)])
    monkeypatch.setenv("SVGD_PHI_SPLIT", split)
    ctxs = {}
    for v in ("1", "0"):
        monkeypatch.setenv("SVGD_X_MIRROR", v)
        ctxs[v] = _ctx(X)
        ctxs[v].diagnostics()
    X2 = oracle.splitmix((n, d), 2.0, 42 + n)
    for step in range(6):
        if step == 3:
            for c in ctxs.values():
                c.set_particles(X2)
        for c in ctxs.values():
            c.step_with_model(model)
        assert np.array_equal(ctxs["1"].get_particles(), ctxs["0"].get_particles()), step
    # steps 1, 2, 4, 5 read the mirror (step 0 and the step after
    # set_particles copy X_t down)
    # (a redone speculative step would copy instead: at most 4)
    assert 3 <= ctxs["1"].diagnostics()["mirror_steps"] <= 4
    assert ctxs["0"].diagnostics()["mirror_steps"] == 0
    for c in ctxs.values():
        c.close()


@pytest.mark.parametrize("n,d", [(3000, 4), (9000, 8)])
def test_resumed_run_matches_uninterrupted(oracle, n, d):
    """A run interrupted by get_particles / set_particles (a checkpoint and
    resume) against the same steps uninterrupted.  The resumed step centres
    with k_mean_partial's mean partials where the uninterrupted one takes the
    previous update's column sums (one launch fewer): the two
    sum in another order, so the mean -- and from there the trajectory --
    may differ in the last bits (INTEGRATION.md "Reproducibility").  Bar:
    positions <= 1e-10, scales rel <= 1e-12."""
    X = oracle.splitmix((n, d), 3.0, 50 + n + d)
    mus = oracle.splitmix((2, d), 2.0, 51)
    model = S.GaussianSum(list(mus), [np.eye(d) * (1.0 + 0.25 * c) for c in range(2)])
    a, b = _ctx(X), _ctx(X)
    for _ in range(6):
        a.step_with_model(model)
    for step in range(6):
        if step == 3:
            b.set_particles(b.get_particles())
        b.step_with_model(model)
    assert a.last_scale()[0] == pytest.approx(b.last_scale()[0], rel=1e-12)
    assert np.max(np.abs(a.get_particles() - b.get_particles())) <= 1e-10
    a.close()
    b.close()
