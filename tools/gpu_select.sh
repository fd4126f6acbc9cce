#!/bin/bash
# Counting select for small buckets: the median tests, then cfg3 / cfg2 /
# sim-world 8 lines and the cfg2 timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
source tools/fault_guard.sh
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_median_paths.py tests/test_gpu_speculative.py tests/test_gpu_track.py tests/test_gpu_collect.py tests/test_gpu_multirank.py tests/test_gpu_fullsize.py tests/test_gpu_rccl.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_sel.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/ab/pytest_sel.log; fault_guard gpurun_out/ab/pytest_sel.log; [ $rc -ne 0 ] && exit $rc
for a in "--config cfg3" "--config cfg2" "--sim-world 8"; do
  timeout -k 10 300 python bench.py $a --steps 20 --warmup 5 --no-cpu > gpurun_out/ab/sel.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print(sys.argv[2], round(d['ms_per_step'],4), [round(x,3) for x in d['repeats']['ms_per_step']], d['phases_ms_per_step'], d['tracked_brackets'], d['gpu_timed']['gfxclk_mhz_median'])" gpurun_out/ab/sel.log "$a"
done
CONFIGS="cfg2" bash tools/gpu_timeline.sh
