#!/bin/bash
# Polled selection completion (no status event): median/step tests, then A/B
# against the event (SVGD_STATUS_POLL=0) at cfg2 / sim-world 8 / cfg3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
source tools/fault_guard.sh
timeout -k 10 900 python -u -m pytest tests/test_gpu_speculative.py tests/test_gpu_track.py tests/test_gpu_median_paths.py tests/test_gpu_parity.py tests/test_gpu_host_model_step.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_poll.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab/pytest_poll.log; fault_guard gpurun_out/ab/pytest_poll.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="base SVGD_STATUS_POLL=0" BENCH_ARGS="--config cfg2" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
VARIANTS="base SVGD_STATUS_POLL=0" BENCH_ARGS="--sim-world 8" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
VARIANTS="base SVGD_STATUS_POLL=0" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
CONFIGS="cfg2" bash tools/gpu_timeline.sh
