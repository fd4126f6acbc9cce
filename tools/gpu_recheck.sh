#!/bin/bash
# The driver's round-end commands once more on another box: smoke, the GPU
# suite, the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
mkdir -p gpurun_out/recheck
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/recheck/smoke.log 2>&1 || { tail -5 gpurun_out/recheck/smoke.log; exit 1; }
tail -1 gpurun_out/recheck/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/recheck/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/recheck/pytest_gpu.log; fault_guard gpurun_out/recheck/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/recheck/bench_default.log 2>&1 || { tail -5 gpurun_out/recheck/bench_default.log; exit 1; }
tail -1 gpurun_out/recheck/bench_default.log | cut -c1-400
