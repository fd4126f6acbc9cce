#!/bin/bash
# Column-split 8-wave phi kernel (default kind 2): parity, A/B against the
# 4-wave kernel and split multipliers (cfg3, cfg2), sim-world P = 2, 4, 8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
source tools/fault_guard.sh
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_speculative.py tests/test_gpu_sym.py tests/test_gpu_multirank.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_wc.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/ab/pytest_wc.log; fault_guard gpurun_out/ab/pytest_wc.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="base SVGD_PHI_T8K=0 SVGD_PHI_SPLIT_MULT=1 SVGD_PHI_SPLIT_MULT=4" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
VARIANTS="base SVGD_PHI_T8K=0" BENCH_ARGS="--config cfg2" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
WORLDS="2 4 8" MULTS="1 4" bash tools/gpu_sim_world.sh
