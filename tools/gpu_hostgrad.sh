#!/bin/bash
# Host gradient rework (vector mixture weights / combination): the host-model
# and device-model tests, the sharded tracking test, then cfg3 / cfg2 lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
source tools/fault_guard.sh
timeout -k 10 900 python -u -m pytest tests/test_gpu_host_model_step.py tests/test_gpu_device_model.py tests/test_gpu_multirank.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_hg.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/ab/pytest_hg.log; fault_guard gpurun_out/ab/pytest_hg.log; [ $rc -ne 0 ] && exit $rc
for cfg in cfg3 cfg2; do
  timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu > gpurun_out/ab/hg_$cfg.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print(sys.argv[1], d['ms_per_step'], d['repeats']['ms_per_step'], d['host_ms_per_step'], d['diag_ms_per_step'], d['phases_ms_per_step'], d['gpu_timed']['gfxclk_mhz_median'])" gpurun_out/ab/hg_$cfg.log
done
