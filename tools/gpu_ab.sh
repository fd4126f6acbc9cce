#!/bin/bash
# GPU iteration: parity tests, then cfg3 and cfg2 bench lines (no CPU leg).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
source tools/fault_guard.sh
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
fault_guard gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for cfg in cfg3 cfg2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --config $cfg ${BENCH_ARGS:-} > gpurun_out/bench_$cfg.log 2>&1 || exit $?
  fault_guard gpurun_out/bench_$cfg.log
  tail -1 gpurun_out/bench_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['ms_per_step'], d['phases_ms_per_step'], d['roofline']['frac'])"
done
