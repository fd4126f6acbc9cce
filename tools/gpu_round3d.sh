#!/bin/bash
# Bracket tracking: parity (bit-identical trajectories), A/B against sampled
# brackets at cfg3 / cfg2 / sim-world 8; per-lane below counters in k_pair_mcol
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
source tools/fault_guard.sh
timeout -k 10 900 python -u -m pytest tests/test_gpu_track.py tests/test_gpu_speculative.py tests/test_gpu_median_paths.py tests/test_gpu_multirank.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_trk.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/ab/pytest_trk.log; fault_guard gpurun_out/ab/pytest_trk.log; [ $rc -ne 0 ] && exit $rc
SVGD_MCOL_VCOUNT=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_collect.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_vcount.log 2>&1; rc=$?
echo "pytest vcount rc=$rc"; tail -3 gpurun_out/ab/pytest_vcount.log; fault_guard gpurun_out/ab/pytest_vcount.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="base SVGD_TRACK_BRACKET=0 SVGD_MCOL_VCOUNT=1" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
VARIANTS="base SVGD_TRACK_BRACKET=0 SVGD_MCOL_VCOUNT=1" BENCH_ARGS="--config cfg2" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
VARIANTS="base SVGD_TRACK_BRACKET=0" BENCH_ARGS="--sim-world 8" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
for f in gpurun_out/ab/base.1.log gpurun_out/ab/base.1--config_cfg2.log gpurun_out/ab/base.1--sim-world_8.log; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print(sys.argv[1], d['tracked_brackets'], d['phases_ms_per_step'])" $f
done
CONFIGS="cfg3" BENCH_ARGS="" bash tools/gpu_timeline.sh
SVGD_MCOL_VCOUNT=1 CONFIGS="cfg2" bash tools/gpu_timeline.sh
