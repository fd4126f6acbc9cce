#!/bin/bash
# Band staging forms (SVGD_MCOL_STAGE 0 / 1 / 2 as tools/ablibs/code, st1, st2;
# the library in place is the candidate): bit-exact collect tests, then
# k_pair_mcol time per form and the step time
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
source tools/fault_guard.sh
timeout -k 10 600 python -u -m pytest tests/test_gpu_collect.py tests/test_gpu_fullsize.py tests/test_gpu_median_paths.py tests/test_gpu_track.py tests/test_gpu_speculative.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_stage.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab/pytest_stage.log; fault_guard gpurun_out/ab/pytest_stage.log; [ $rc -ne 0 ] && exit $rc
ROUNDS=2 bash tools/gpu_mcol_abl.sh code st1 st2 || exit 1
CFG=cfg2 bash tools/gpu_mcol_abl.sh code st1 st2 || exit 1
ROUNDS=2 bash tools/ab_libs.sh code st1 st2 || exit 1
