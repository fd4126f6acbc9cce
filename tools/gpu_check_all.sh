#!/bin/bash
# The whole GPU suite, smoke, then cfg3 / cfg2 / sim-world 8 lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
source tools/fault_guard.sh
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_all.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab/pytest_all.log; fault_guard gpurun_out/ab/pytest_all.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ab/smoke.log 2>&1 || { tail -5 gpurun_out/ab/smoke.log; exit 1; }
tail -1 gpurun_out/ab/smoke.log
for a in "--config cfg3" "--config cfg2" "--sim-world 8"; do
  timeout -k 10 300 python bench.py $a --steps 20 --warmup 5 --no-cpu > gpurun_out/ab/chk.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print(sys.argv[2], round(d['ms_per_step'],4), [round(x,3) for x in d['repeats']['ms_per_step']], d['phases_ms_per_step'], d['tracked_brackets'], d['gpu_timed']['gfxclk_mhz_median'], d['roofline']['avg_launch_ms'])" gpurun_out/ab/chk.log "$a"
done
CONFIGS="cfg2" bash tools/gpu_timeline.sh
