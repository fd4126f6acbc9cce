"""World-size-2 (and 3) gloo rehearsal of the sharded SVGD step on CPU.

The library's multi-GPU step shards rows with svgd_plan_rows,
splits median pair tiles with svgd_plan_pair_tiles, brackets the median from
a sharded sample (two histogram all-reduces), all-reduces the counts + bucket
histogram once, all-gathers the selected buckets' keys once (or, after a
bracket miss, runs the per-digit radix fallback) and all-gathers X and G.
tests/_multirank_worker.py runs that protocol with gloo in place of RCCL and
numpy/the oracle as the arithmetic; the result must equal the single-process
oracle step.
"""
import multiprocessing as mp
import socket

import numpy as np
import pytest

import _multirank_worker as W


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,n,d,block,sample,sigma,shift,path", [
    (2, 301, 3, 64, 4096, 3.0, 0.0, "bracket"),
    (2, 64, 2, 64, 512, 3.0, 0.0, "bracket"),
    (3, 700, 5, 256, 4096, 3.0, 0.0, "bracket"),
    (4, 900, 8, 256, 8192, 3.0, 0.0, "bracket"),
    (3, 700, 5, 256, 4096, 3.0, 20.0, "fallback"),
])
def test_sharded_step_matches_single_process(oracle, world, n, d, block, sample, sigma, shift, path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=W.run, args=(r, world, port, n, d, block, q, sample, sigma, shift))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        status, res = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert status == "ok", res
    for p in procs:
        assert p.exitcode == 0

    X, mus, covs = res["X"], res["mus"], res["covs"]
    # every unordered pair was keyed by exactly one rank
    assert res["total"] == n * (n - 1) // 2
    # G all-gather reassembles the full matrix bit-for-bit
    np.testing.assert_array_equal(res["G_all"], oracle.logp_grad_gmm(X, mus, covs))
    assert res["path"] == path
    # bracket path: 2 sample-histogram all-reduces + 1 counts all-reduce + 1 key all-gather
    if path == "bracket":
        assert res["collectives"] == 4
    # distributed exact median == single-process median (difference form vs Gram form)
    a_ref, med_ref = oracle.median_scale(X)
    assert res["med"] == pytest.approx(med_ref, rel=1e-13)
    # the sharded step == the single-process step (same a, same rows)
    G = oracle.logp_grad_gmm(X, mus, covs)
    ph = oracle.phi(X, G, res["a"])
    opt = oracle.Adam((n, d), 0.1, 0.9, 0.999)
    X_ref = X.copy()
    oracle.apply_update(X_ref, opt.step(ph), -np.full(d, 2.0), np.full(d, 2.0))
    np.testing.assert_array_equal(res["X_new"], X_ref)
