#!/bin/bash
# Round 5: the row-stream hand-over of the symmetric pass without its reduce
# launch (finish / apply sum its partials) -- symmetric, sharded and parity
# GPU tests, then cfg3 step timelines at P = 1 and the P = 4 / 8 shares.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r5o
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_gpu_sym.py tests/test_gpu_parity.py tests/test_gpu_rccl.py "tests/test_gpu_multirank.py::test_sharded_symmetric_phi" > $O/pytest.log 2>&1
rc=$?; fault_guard $O/pytest.log; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "^FAILED|Error" $O/pytest.log | head; exit 1; }
VARIANTS="p1:-" bash tools/gpu_tl_var.sh || exit 1
VARIANTS="sim4:- sim8sym:SVGD_PHI_SYM=1" BENCH_ARGS="--sim-world 4" bash tools/gpu_tl_var.sh > /dev/null || exit 1
echo "== sim4"; cat gpurun_out/tlvar/sim4.txt
VARIANTS="sim8sym:SVGD_PHI_SYM=1" BENCH_ARGS="--sim-world 8" bash tools/gpu_tl_var.sh || exit 1
echo r5o done
