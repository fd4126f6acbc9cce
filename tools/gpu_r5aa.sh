#!/bin/bash
# Round 5: centring with shuffle trees (c1) vs LDS trees (c0): GPU tests that
# pin the centring (parity, speculative redo, resume, multi-rank), cfg3 and
# sim-8 timelines, same-box A/B lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
mkdir -p gpurun_out/r5aa
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_speculative.py tests/test_gpu_host_model_step.py tests/test_gpu_multirank.py tests/test_gpu_sym.py > gpurun_out/r5aa/pytest.log 2>&1
rc=$?; fault_guard gpurun_out/r5aa/pytest.log; tail -2 gpurun_out/r5aa/pytest.log; [ $rc = 0 ] || { grep -E "^FAILED|Error" gpurun_out/r5aa/pytest.log | head; exit 1; }
VARIANTS="p1:-" bash tools/gpu_tl_var.sh > /dev/null || exit 1
grep -E "k_center|span" gpurun_out/tlvar/p1.txt
VARIANTS="s8:-" BENCH_ARGS="--sim-world 8" bash tools/gpu_tl_var.sh > /dev/null || exit 1
grep -E "k_center|span" gpurun_out/tlvar/s8.txt
ROUNDS=2 bash tools/ab_libs.sh c0 c1 || exit 1
echo r5aa done
