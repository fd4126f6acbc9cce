#!/bin/bash
# Round 5: k_phi_sym with one barrier per sub-tile (b1) vs two (a0): the
# symmetric GPU tests, then same-box alternated cfg3 lines and the P = 4 share.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
mkdir -p gpurun_out/r5w
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_gpu_sym.py "tests/test_gpu_multirank.py::test_sharded_symmetric_phi" tests/test_gpu_rccl.py > gpurun_out/r5w/pytest.log 2>&1
rc=$?; fault_guard gpurun_out/r5w/pytest.log; tail -2 gpurun_out/r5w/pytest.log; [ $rc = 0 ] || exit 1
ROUNDS=3 bash tools/ab_libs.sh ${LIBS:-a0 b1} || exit 1
ROUNDS=2 BENCH_ARGS="--sim-world 4" bash tools/ab_libs.sh ${LIBS:-a0 b1} || exit 1
VARIANTS="p1:-" bash tools/gpu_tl_var.sh > /dev/null || exit 1
grep -E "k_phi_sym|span" gpurun_out/tlvar/p1.txt
echo r5w done
