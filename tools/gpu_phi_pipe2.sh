#!/bin/bash
# Pipelined phi row stream (A(j+1) ; B(j)): GPU parity, then step time and
# phi kernel time against the previous library (tools/ablibs/code.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
source tools/fault_guard.sh
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_speculative.py tests/test_gpu_host_model_step.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_pipe2.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab/pytest_pipe2.log; fault_guard gpurun_out/ab/pytest_pipe2.log; [ $rc -ne 0 ] && exit $rc
ROUNDS=3 bash tools/ab_libs.sh code pipe2 || exit 1
