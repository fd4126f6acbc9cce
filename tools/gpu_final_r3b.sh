#!/bin/bash
# Round-3 final evidence, part 1 (one gpurun call): the driver's own commands
# (smoke, the default bench line), the GPU suite, round_profile.sh (bench line
# with the CPU leg, rocprof stats and steady-state kernel means of the same
# command, step timeline, FETCH_SIZE / WRITE_SIZE passes, cfg5 / cfg2 lines)
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
source tools/fault_guard.sh
mkdir -p gpurun_out/round
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round/smoke.log 2>&1 || { tail -5 gpurun_out/round/smoke.log; exit 1; }
tail -1 gpurun_out/round/smoke.log
start=$(date +%s)
timeout -k 10 600 python bench.py > gpurun_out/round/bench_default.log 2>&1 || { tail -5 gpurun_out/round/bench_default.log; exit 1; }
echo "default bench took $(( $(date +%s) - start )) s"
tail -1 gpurun_out/round/bench_default.log > gpurun_out/round/bench_default.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/round/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/round/pytest_gpu.log; fault_guard gpurun_out/round/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
bash tools/round_profile.sh || exit 1
echo part1 done
