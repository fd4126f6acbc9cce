#!/bin/bash
# Round-3 GPU session: the -m gpu suite (one process, per-test timeout), smoke,
# the headline bench line and the cfg2 line.  Each GPU step has its own
# limit; a fault, abort or timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
source tools/fault_guard.sh
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
fault_guard gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
fault_guard gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-600
fault_guard gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config cfg2 --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_cfg2.log 2>&1
rc=$?; echo "bench cfg2 rc=$rc"; tail -1 gpurun_out/bench_cfg2.log | cut -c1-400
fault_guard gpurun_out/bench_cfg2.log
exit $rc
