#!/bin/bash
# Tracked brackets on the tile paths: parity, then cfg5 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
source tools/fault_guard.sh
timeout -k 10 900 python -u -m pytest tests/test_gpu_track.py tests/test_gpu_median_paths.py tests/test_gpu_f32.py tests/test_gpu_speculative.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_trk_tile.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/ab/pytest_trk_tile.log; fault_guard gpurun_out/ab/pytest_trk_tile.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="base SVGD_TRACK_BRACKET=0" BENCH_ARGS="--config cfg5" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print(d['tracked_brackets'], d['phases_ms_per_step'])" "gpurun_out/ab/base.1--config_cfg5.log"
