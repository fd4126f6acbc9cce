"""The sharded symmetric phi pass's protocol on CPU with gloo, world 1-4
(tests/_sym_exchange_worker.py): the ranks' units (svgd_plan_sym_units) must
cover every unordered pair of particles exactly once off the diagonal tiles
and every ordered pair inside them, every sum a rank produces lies in the
ranges svgd_plan_sym_exchange plans, and the point-to-point exchanged
per-particle sums give each rank the single-process phi_hat of its rows
(oracle, SVGD.hpp:407-454) -- 1e-12 relative (a different summation
order)."""
import multiprocessing as mp
import socket

import numpy as np
import pytest

import _sym_exchange_worker as W


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,n,d,block", [(1, 300, 3, 64), (2, 500, 3, 64), (3, 777, 2, 128), (4, 1000, 8, 192),
                                             (8, 2000, 2, 64), (8, 1537, 3, 128), (6, 3000, 2, 192)])
def test_sym_exchange_matches_oracle(oracle, world, n, d, block):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    a = 0.31
    procs = [ctx.Process(target=W.run, args=(r, world, port, n, d, block, a, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        status, res = q.get(timeout=300)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert status == "ok", res
    nb = (n + block - 1) // block
    # the units' pairs: every off-diagonal block pair once, every diagonal square whole
    diag = sum(min(block, n - I * block) ** 2 for I in range(nb))
    assert res["pairs"] == (n * n - diag) // 2 + diag
    ref = oracle.phi(res["X"], res["G"], a)
    got = np.zeros_like(ref)
    for r0, r1, ph in res["rows"]:
        got[r0:r1] = ph
    scale = np.max(np.abs(ref))
    assert np.max(np.abs(got - ref)) <= 1e-12 * scale
