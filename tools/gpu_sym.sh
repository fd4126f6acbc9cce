#!/bin/bash
# Symmetric phi pass: parity tests, then interleaved A/B bench lines (cfg3, cfg2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
source tools/fault_guard.sh
timeout -k 10 600 python -u -m pytest tests/test_gpu_sym.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_sym.log 2>&1
rc=$?; echo "pytest sym rc=$rc"; grep -E "passed|failed|Error|error" gpurun_out/ab/pytest_sym.log | tail -5
fault_guard gpurun_out/ab/pytest_sym.log
[ $rc -ne 0 ] && exit $rc
VARIANTS="base SVGD_PHI_SYM=1" bash tools/gpu_ab_phi.sh 2>&1 | grep -v "^pytest\|passed"
VARIANTS="base SVGD_PHI_SYM=1" BENCH_ARGS="--config cfg2" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh
