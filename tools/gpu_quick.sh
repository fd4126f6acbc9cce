#!/bin/bash
# Quick GPU iteration: parity tests, one bench line (no CPU leg), kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
source tools/fault_guard.sh
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
fault_guard gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu ${BENCH_ARGS:-} > gpurun_out/bench_quick.log 2>&1 || exit $?
fault_guard gpurun_out/bench_quick.log
tail -1 gpurun_out/bench_quick.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['phases_ms_per_step'], d['roofline']['frac'])"
STEPS=5 TAG=${TAG:-_quick} bash tools/profile.sh > /dev/null && python3 tools/kstats.py gpurun_out/prof${TAG:-_quick}/run_kernel_stats.csv | head -8
