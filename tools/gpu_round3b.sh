#!/bin/bash
# check_b16, the 8K-table phi A/B (cfg3, cfg2), sim-world P = 2, 4, 8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
timeout -k 10 60 ./tools/check_b16 || exit 1
VARIANTS="base SVGD_PHI_T8K=1" bash tools/gpu_ab_phi.sh 2>&1 | grep -v "^pytest\|passed" || exit 1
VARIANTS="base SVGD_PHI_T8K=1" BENCH_ARGS="--config cfg2" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
timeout -k 10 600 env SVGD_PHI_T8K=1 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_speculative.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_t8k.log 2>&1; rc=$?
echo "pytest t8k rc=$rc"; tail -1 gpurun_out/ab/pytest_t8k.log; fault_guard gpurun_out/ab/pytest_t8k.log; [ $rc -ne 0 ] && exit $rc
WORLDS="2 4 8" MULTS="" bash tools/gpu_sim_world.sh
