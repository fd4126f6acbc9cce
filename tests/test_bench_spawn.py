"""bench.py --gpus N without a launcher (spawn_ranks): the ranks are polled,
and the first one that fails ends the others, so a dead rank cannot leave
the rest blocked in RCCL until an outside timeout with no line written.
CPU only (stand-in ranks: tests/_spawn_child.py)."""
import os
import time

import bench

CHILD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_spawn_child.py")


def test_spawn_ranks_all_succeed(monkeypatch):
    monkeypatch.setenv("SLEEP", "0.2")
    monkeypatch.delenv("FAIL_RANK", raising=False)
    assert bench.spawn_ranks(3, argv=[CHILD]) == 0


def test_spawn_ranks_first_failure_ends_the_others(monkeypatch):
    monkeypatch.setenv("SLEEP", "120")
    monkeypatch.setenv("FAIL_RANK", "1")
    t0 = time.time()
    rc = bench.spawn_ranks(4, argv=[CHILD], grace=5.0)
    assert rc == 3
    assert time.time() - t0 < 30  # not the sleepers' 120 s
