"""The RCCL collectives of the sharded step, executed on one GPU.

A context created with world = 1 and an RCCL unique id owns a one-rank RCCL
communicator, so every collective call site of the multi-GPU step runs through
RCCL (ncclCommInitRank, in-place ncclAllGather of X and G, ncclAllReduce of the
bracket-sample histograms, of the median counts + bucket histogram and, on the
fallback path, of each radix digit; ncclAllGather of the selected-bucket keys).
RCCL refuses two ranks on one device, so this is the most of the RCCL path a
one-GPU box can run; the multi-rank protocol itself is covered by
tests/test_gpu_multirank.py (host shared-memory collectives, same call sites)
and tests/test_multirank_cpu.py (gloo).

Bar: bit-identical to the same steps without a communicator (a one-rank sum
or gather is the identity), on the bracket, bucket-select and forced radix
fallback paths.  GPU only."""
import numpy as np
import pytest

import svgdcpp_amd as S
from svgdcpp_amd import _capi as C

pytestmark = pytest.mark.gpu


def _run(oracle, n, d, steps, rccl, monkeypatch, bucket_cap=None, sample=None, diag=None):
    if bucket_cap is not None:
        monkeypatch.setenv("SVGD_BUCKET_CAP", str(bucket_cap))
    uid = S.Context.unique_id() if rccl else None
    c = S.Context(d, n, world=1, rank=0, unique_id=uid)
    X0 = oracle.splitmix((n, d), 3.0, 71)
    mus = oracle.splitmix((4, d), 3.0, 72)
    model = S.GaussianSum(list(mus), [np.eye(d) * (1.0 + 0.25 * k) for k in range(4)])
    c.set_particles(X0)
    c.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999, 1e-8)
    if sample:
        c.check(c.lib.svgd_set_median_tuning(c.h, -1, sample, -1))
    if diag is not None:
        c.diagnostics()
        c.check(c.lib.svgd_set_timing(c.h, 2))  # count the collectives
    scales = []
    for _ in range(steps):
        c.step_with_model(model)
        scales.append(c.last_scale())
    X = c.get_particles()
    if diag is not None:
        diag.update(c.diagnostics())
        c.check(c.lib.svgd_set_timing(c.h, 0))
    c.close()
    return X, scales


@pytest.mark.parametrize("n,d,bucket_cap", [(6000, 8, None), (6000, 8, 0), (3000, 2, None), (700, 24, None)])
def test_rccl_one_rank_step_bit_identical(oracle, monkeypatch, n, d, bucket_cap):
    Xa, sa = _run(oracle, n, d, 3, True, monkeypatch, bucket_cap)
    Xb, sb = _run(oracle, n, d, 3, False, monkeypatch, bucket_cap)
    assert sa == sb
    assert np.array_equal(Xa, Xb)
    if n * (n - 1) // 2 > (1 << 24):
        assert all(s[2] in (C.SVGD_MEDIAN_BRACKET, C.SVGD_MEDIAN_REBRACKET, C.SVGD_MEDIAN_FALLBACK)
                   for s in sa)


def test_rccl_one_rank_tracked_brackets(oracle, monkeypatch):
    """16 steps through the one-rank RCCL communicator (every collective on
    the compute stream, tracked median brackets from the fourth speculative
    step on) against the same steps without one: bit-identical."""
    dg = {}
    Xa, sa = _run(oracle, 6000, 8, 16, True, monkeypatch, diag=dg)
    Xb, sb = _run(oracle, 6000, 8, 16, False, monkeypatch)
    assert sa == sb
    assert np.array_equal(Xa, Xb)
    assert dg["ranks"] == 1 and dg["g_comm"] == 0 and dg["gather_g_n"] == 0
    assert dg["coll_n"] >= 16 * 3 and dg["trk_steps"] >= 3


@pytest.mark.parametrize("n,d", [(6000, 8), (700, 24)])
def test_rccl_one_rank_split_g_communicator(oracle, monkeypatch, n, d):
    """SVGD_G_COMM=1: the G all-gather on its own communicator (ncclCommSplit
    of the context's, the split's success agreed by a min all-reduce) and its
    own stream, beside the median chain, the phi chain waiting on its event
    -- 16 steps against the same steps without any communicator:
    bit-identical, and the diagnostics show the split communicator carried
    one G all-gather per step."""
    monkeypatch.setenv("SVGD_G_COMM", "1")
    dg = {}
    Xa, sa = _run(oracle, n, d, 16, True, monkeypatch, diag=dg)
    monkeypatch.delenv("SVGD_G_COMM")
    Xb, sb = _run(oracle, n, d, 16, False, monkeypatch)
    assert sa == sb
    assert np.array_equal(Xa, Xb)
    assert dg["g_comm"] == 1 and dg["ranks"] == 1, dg
    assert dg["gather_g_n"] == 16, dg


def test_rccl_one_rank_symmetric_exchange(oracle, monkeypatch):
    """SVGD_PHI_SYM=2: the sharded symmetric form (every particle's sums from
    the rank's pair units, the exchange's ncclGroupStart / ncclGroupEnd with
    no peer to send to, k_sym_apply) on the one-rank communicator, 6 steps: bit-identical to the same form without a
    communicator and to the one-rank symmetric pass (SVGD_PHI_SYM=1: the same
    partials summed in the same order, phi formed by the same expression)."""
    n, d = 6000, 8
    monkeypatch.setenv("SVGD_PHI_SYM", "2")
    Xa, sa = _run(oracle, n, d, 6, True, monkeypatch)
    Xb, sb = _run(oracle, n, d, 6, False, monkeypatch)
    monkeypatch.setenv("SVGD_PHI_SYM", "1")
    Xc, sc = _run(oracle, n, d, 6, False, monkeypatch)
    assert sa == sb == sc
    assert np.array_equal(Xa, Xb) and np.array_equal(Xa, Xc)
