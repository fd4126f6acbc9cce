#!/bin/bash
# bf16-split Gram in the collect (SVGD_MCOL_BF16=1; tools/ablibs/bf.so has it
# on by default): bit-exact collect / median tests with it on, then
# k_pair_mcol time and step time against the f32 Gram (tools/ablibs/st1.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
source tools/fault_guard.sh
SVGD_MCOL_BF16=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_collect.py tests/test_gpu_fullsize.py tests/test_gpu_median_paths.py tests/test_gpu_track.py tests/test_gpu_speculative.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_bf16.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/ab/pytest_bf16.log; fault_guard gpurun_out/ab/pytest_bf16.log; [ $rc -ne 0 ] && exit $rc
ROUNDS=2 bash tools/gpu_mcol_abl.sh st1 bf || exit 1
CFG=cfg2 bash tools/gpu_mcol_abl.sh st1 bf || exit 1
ROUNDS=2 bash tools/ab_libs.sh st1 bf || exit 1
BENCH_ARGS="--sim-world 8" ROUNDS=1 bash tools/ab_libs.sh st1 bf || exit 1
