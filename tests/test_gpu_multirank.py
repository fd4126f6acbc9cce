"""Sharded step rehearsal on one GPU: world = 2, 3 and 8 ranks on device 0 with
the host shared-memory collective backend (SVGD_HOSTCOMM) vs the same
problem on one rank.  The median is an exact order statistic, so the first
step's scale must agree bit for bit (later steps: to rounding of X_t); phi sums columns in a different split, so positions
agree to fp64 rounding, which Adam's normalised step can amplify where
phi_hat ~ 0: 1e-10 after 4 steps (observed <= 1.3e-12).  The RCCL calls themselves are the same
in-place all-gather / sum all-reduce at the same call sites."""
import multiprocessing as mp
import os
import uuid

import numpy as np
import pytest

import _gpu_rank_worker as W

pytestmark = pytest.mark.gpu


def _run_ranks(world, n, d, steps, env=None, trk=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = "svgd_" + uuid.uuid4().hex[:12]
    procs = [ctx.Process(target=W.run, args=(r, world, name, n, d, steps, q, env)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            status, rank, X, scales, shard, ntrk = q.get(timeout=300)
            assert status == "ok", X
            out[rank] = (X, scales, shard)
            if trk is not None:
                trk[rank] = ntrk
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return out


@pytest.mark.parametrize("world,n", [(2, 3001), (3, 6007), (8, 20011)])
def test_sharded_step_matches_single_rank(world, n):
    d, steps = 5, 4
    multi = _run_ranks(world, n, d, steps)
    single = _run_ranks(1, n, d, steps)[0]
    X1, s1, _ = single
    shards = sorted(v[2] for v in multi.values())
    assert shards[0][0] == 0 and shards[-1][1] == n  # rows partition [0, n)
    for (a0, a1), (b0, b1) in zip(shards, shards[1:]):
        assert a1 == b0
    for rank, (X, scales, _) in multi.items():
        # every rank holds the all-gathered particles; the first step's scale
        # (same X_0) is bit-identical to one rank's, later ones follow X_t,
        # which differs from one rank's in the last bits (phi splits)
        assert scales[0][0] == s1[0][0], (rank, scales, s1)
        np.testing.assert_allclose([s[0] for s in scales], [s[0] for s in s1], rtol=1e-13)
        assert [s[2] for s in scales] == [s[2] for s in s1]
        np.testing.assert_allclose(X, X1, rtol=0, atol=1e-10)


@pytest.mark.parametrize("world,n", [(2, 12007), (8, 20011)])
def test_sharded_tracked_brackets_bit_identical(world, n):
    """The tracked median bracket on a sharded run: every rank predicts the
    same bracket from the same all-reduced counts and selected keys, and the
    trajectory is bit-identical to sampling every bracket."""
    d, steps = 5, 14
    trk = {}
    tracked = _run_ranks(world, n, d, steps, {"SVGD_TRACK_BRACKET": "1"}, trk)
    sampled = _run_ranks(world, n, d, steps, {"SVGD_TRACK_BRACKET": "0"})
    assert min(trk.values()) >= 3 and len(set(trk.values())) == 1
    for rank in range(world):
        Xa, sa, _ = tracked[rank]
        Xb, sb, _ = sampled[rank]
        assert np.array_equal(Xa, Xb), rank
        assert sa == sb, rank
