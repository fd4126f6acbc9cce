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


def _run_ranks(world, n, d, steps, env=None, trk=None, diags=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = "svgd_" + uuid.uuid4().hex[:12]
    procs = [ctx.Process(target=W.run, args=(r, world, name, n, d, steps, q, env)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            status, rank, X, scales, shard, diag = q.get(timeout=300)
            assert status == "ok", X
            out[rank] = (X, scales, shard)
            if trk is not None:
                trk[rank] = diag["trk_steps"]
            if diags is not None:
                diags[rank] = diag
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return out


@pytest.mark.parametrize("world,n", [(2, 3001), (3, 6007), (8, 20011)])
def test_sharded_step_matches_single_rank(world, n):
    d, steps = 5, 4
    # SVGD_DEBUG_COLL: every step all-gathers each rank's hash of its
    # collective sequence and fails on a mismatch (svgd_ctx issue order)
    multi = _run_ranks(world, n, d, steps, {"SVGD_DEBUG_COLL": "1"})
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


@pytest.mark.parametrize("world,n,split", [(4, 12007, "auto"), (8, 20011, "auto"), (4, 12007, "1"),
                                           (8, 20011, "1")])
def test_default_multirank_path_row_parts(world, n, split):
    """The path a rank of P >= 4 takes at cfg3: the next
    gradient reading the update's pinned X mirror, speculative steps with
    tracked median brackets, every step's collective sequence hashed and
    compared across ranks (SVGD_DEBUG_COLL=1) -- with phi + update whole
    (split "auto": the policy's choice at SVGD_HOST_THREADS=1, a rank of 8 on
    a 16-CPU box has 2 threads) and in two row parts (SVGD_PHI_SPLIT=1, the
    first part's X_{t+1} feeding the gradient early) -- against one rank of
    the same problem: the first scale bit-exact, later ones to the rounding of
    X_t (1e-13), positions <= 1e-10 (phi's column splits differ)."""
    d, steps = 5, 10
    diags = {}
    env = {"SVGD_HOST_THREADS": "1", "SVGD_DEBUG_COLL": "1"}
    if split != "auto":
        env["SVGD_PHI_SPLIT"] = split
    multi = _run_ranks(world, n, d, steps, env, diags=diags)
    single = _run_ranks(1, n, d, steps, {"SVGD_HOST_THREADS": "1"})[0]
    X1, s1, _ = single
    for rank, (X, scales, (r0, r1)) in multi.items():
        dg = diags[rank]
        assert dg["ranks"] == world, dg
        # forced split: every step but a redone one (a redo runs phi whole)
        # in row parts; all but the first read X_t from the mirror; tracked
        # brackets
        if split == "1":
            assert dg["split_steps"] >= steps - 2, (rank, dg)
        assert dg["mirror_steps"] >= steps - 3, (rank, dg)
        assert dg["spec_steps"] >= steps - 3 and dg["trk_steps"] >= 3, (rank, dg)
        assert scales[0][0] == s1[0][0], (rank, scales, s1)
        np.testing.assert_allclose([s[0] for s in scales], [s[0] for s in s1], rtol=1e-13)
        np.testing.assert_allclose(X, X1, rtol=0, atol=1e-10)
    # the ranks' trajectories are one trajectory
    Xs = [multi[r][0] for r in range(world)]
    assert all(np.array_equal(Xs[0], x) for x in Xs[1:])
    assert len({tuple(s[0] for s in multi[r][1]) for r in range(world)}) == 1


@pytest.mark.parametrize("world,n,d", [(2, 3001, 5), (3, 6007, 8), (4, 12007, 2), (8, 30011, 3), (6, 20011, 8)])
def test_sharded_symmetric_phi(world, n, d):
    """The symmetric phi pass sharded (SVGD_PHI_SYM=1 at P > 1): rank r runs
    the pair units [U r / P, U (r+1) / P), sums every particle's partials from
    them, and the point-to-point exchange (svgd_plan_sym_exchange; the host
    backend delivers only what the senders sent, NaN elsewhere) hands each
    rank its rows' pieces for k_sym_apply -- against one rank on the row
    stream: the first scale bit-exact, positions <= 1e-10 (the pair sums are
    grouped differently, fp64 rounding)."""
    steps = 4
    diags = {}
    multi = _run_ranks(world, n, d, steps, {"SVGD_PHI_SYM": "1", "SVGD_DEBUG_COLL": "1"}, diags=diags)
    single = _run_ranks(1, n, d, steps, {"SVGD_PHI_SYM": "0"}, diags=(d1 := {}))[0]
    assert d1[0]["phi_kernel"].startswith("k_phi_rows"), d1
    X1, s1, _ = single
    for rank, (X, scales, _) in multi.items():
        assert diags[rank]["phi_kernel"].startswith("k_phi_sym"), diags[rank]
        assert scales[0][0] == s1[0][0], (rank, scales, s1)
        np.testing.assert_allclose([s[0] for s in scales], [s[0] for s in s1], rtol=1e-13)
        np.testing.assert_allclose(X, X1, rtol=0, atol=1e-10)
    Xs = [multi[r][0] for r in range(world)]
    assert all(np.array_equal(Xs[0], x) for x in Xs[1:])


def _sample_rows(n):
    # both ends and 512 rows straddling n / 2 (a rank boundary at P = 8: the
    # rows of two ranks, each from its own exchange)
    return [(0, 256), (n // 2 - 256, n // 2 + 256), (n - 256, n)]


@pytest.mark.parametrize("n,sym", [(131072, "default"), (65536, "default"), (65536, "0")],
                         ids=["n131072-sym-default", "cfg3-sym-default", "cfg3-rows-forced"])
def test_world8_full_path_vs_one_rank_and_oracle(oracle, n, sym):
    """8 ranks at d = 8 through the default multi-rank path (X mirror,
    speculative steps, tracked brackets, SVGD_DEBUG_COLL=1).  n = 131072:
    N/P = 16384 rows per rank makes the sharded symmetric pass the default
    (cfg4's 8-rank form at half its N); n = 65536: cfg3's 8-rank default
    (the sharded symmetric pass from N/P >= 8192) and the row stream forced.  The host backend's
    phi exchange is a faithful point-to-point one -- a receiver sees only the
    ranges its senders sent (NaN elsewhere) and a range the two sides plan
    differently fails the call -- so a rank reading sums it was not sent
    fails here.  Checks:
    the first scale bit-exact vs one rank, later ones to X_t's rounding,
    positions <= 1e-10 vs one rank, the 8 ranks' trajectories identical, and
    one more sharded phi of X_T on 1024 sampled rows (both ends and a rank
    boundary) against the oracle's phi of the all-gathered X_T: <= 1e-10."""
    d, steps, world = 8, 10, 8
    env = {"SVGD_DEBUG_COLL": "1", "SVGD_HOST_THREADS": "1", "TEST_PHI_CHECK": "1"}
    if sym != "default":
        env["SVGD_PHI_SYM"] = sym
    diags = {}
    multi = _run_ranks(world, n, d, steps, env, diags=diags)
    single = _run_ranks(1, n, d, steps, {"SVGD_HOST_THREADS": "1"})[0]
    X1, s1, _ = single
    want_sym = sym != "0" and n // world >= 8192
    for rank, (X, scales, _) in multi.items():
        dg = diags[rank]
        assert dg["ranks"] == world, dg
        assert dg["phi_kernel"].startswith("k_phi_sym" if want_sym else "k_phi_rows"), dg["phi_kernel"]
        # (the bracket is tracked once the last medians predict it closely:
        # the first steps of a fresh trajectory move fast)
        assert dg["spec_steps"] >= steps - 3 and dg["trk_steps"] >= 1, (rank, dg)
        assert scales[0][0] == s1[0][0], (rank, scales, s1)
        np.testing.assert_allclose([s[0] for s in scales], [s[0] for s in s1], rtol=1e-13)
        np.testing.assert_allclose(X, X1, rtol=0, atol=1e-10)
    Xs = [multi[r][0] for r in range(world)]
    assert all(np.array_equal(Xs[0], x) for x in Xs[1:])
    # the extra phi of X_T: every rank's rows, assembled in row order
    XT = Xs[0]
    a = diags[0]["phi_a"]
    assert all(diags[r]["phi_a"] == a for r in range(world))
    ph = np.concatenate([diags[r]["phi_rows"] for r in sorted(diags, key=lambda r: multi[r][2][0])])
    assert ph.shape == (n, d) and np.all(np.isfinite(ph))
    import oracle as O
    mus = O.splitmix((3, d), 3.0, 42)
    import svgdcpp_amd as S
    model = S.GaussianSum(list(mus), [np.eye(d) * (1.0 + 0.25 * c) for c in range(3)])
    G = model.log_model_grad(XT)
    for r0, r1 in _sample_rows(n):
        ref = oracle.phi(XT, G, a, rows=(r0, r1))
        assert np.max(np.abs(ph[r0:r1] - ref)) <= 1e-10, (r0, r1)


def test_sharded_symmetric_phi_hands_over_to_row_stream():
    """Far outliers at P > 1 (a log2e max|xc|^2 > 300 on every rank: the
    flag derives from the all-gathered X): the symmetric form's record prep
    hands the step to the row stream, whose partials k_sym_apply sums -- the
    exchange is still issued (the ranks' sequences never depend on
    device data, SVGD_DEBUG_COLL=1) -- against one rank on the row stream."""
    world, n, d, steps = 3, 6007, 8, 3
    env = {"SVGD_TEST_OUTLIERS": "60", "SVGD_DEBUG_COLL": "1"}
    multi = _run_ranks(world, n, d, steps, dict(env, SVGD_PHI_SYM="1"))
    single = _run_ranks(1, n, d, steps, dict(env, SVGD_PHI_SYM="0"))[0]
    X1, s1, _ = single
    for rank, (X, scales, _) in multi.items():
        assert scales[0][0] == s1[0][0], (rank, scales, s1)
        np.testing.assert_allclose(X, X1, rtol=0, atol=1e-10)


def test_measurement_context_refuses_results():
    """svgd_create_sim (bench.py --sim-world): rank 0's share of a P-rank step,
    measurement only -- it steps, but every call that hands results back
    raises, and the diagnostics name the simulated world and the quota."""
    import svgdcpp_amd as S
    from svgdcpp_amd import _capi as C

    n, d = 4096, 4
    X0 = np.random.default_rng(3).standard_normal((n, d))
    ctx = S.Context(d, n, sim_world=4)
    ctx.set_particles(X0)
    ctx.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999, 1e-8)
    assert (ctx.row0, ctx.row1) == (0, n // 4)
    model = S.GaussianSum([np.zeros(d)], [np.eye(d)])
    ctx.step_with_model(model)
    ctx.sync()
    for call in (ctx.get_particles, ctx.median_scale, lambda: ctx.phi(np.zeros((n // 4, d)), 1.0)):
        with pytest.raises(Exception, match="measurement context"):
            call()
    dg = ctx.diagnostics()
    assert dg["sim_world"] == 4
    if dg["cpu_quota"] > 0:
        # rank 0 of a 4-GPU node: the node's quota is 4 x this box's (CPUs
        # are leased per GPU), so its share is this box's whole quota
        assert dg["host_threads"] <= dg["cpu_quota"]
    ctx.close()


def test_finish_step_needs_begin_step():
    """svgd_finish_step without svgd_begin_step fails before any collective."""
    import svgdcpp_amd as S
    from svgdcpp_amd import _capi as C

    n, d = 512, 3
    ctx = S.Context(d, n)
    ctx.set_particles(np.random.default_rng(4).standard_normal((n, d)))
    ctx.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999, 1e-8)
    G = np.zeros((n, d))
    with pytest.raises(Exception, match="without svgd_begin_step"):
        ctx.check(ctx.lib.svgd_finish_step(ctx.h, C.dptr(G)))
    ctx.close()
