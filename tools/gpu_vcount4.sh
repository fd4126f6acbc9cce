#!/bin/bash
# k_pair_mcol with 4 independent per-lane below counters (SVGD_MCOL_VCOUNT=1): collect tests, A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
source tools/fault_guard.sh
SVGD_MCOL_VCOUNT=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_collect.py tests/test_gpu_fullsize.py tests/test_gpu_track.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_vc4.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab/pytest_vc4.log; fault_guard gpurun_out/ab/pytest_vc4.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="base SVGD_MCOL_VCOUNT=1" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
VARIANTS="base SVGD_MCOL_VCOUNT=1" BENCH_ARGS="--config cfg2" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
SVGD_MCOL_VCOUNT=1 CONFIGS="cfg3" bash tools/gpu_timeline.sh
