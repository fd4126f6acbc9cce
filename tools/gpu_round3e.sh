#!/bin/bash
# Biased-exponent row stream (24 VALU / pair-row) + the predicted bracket's
# state written by the centring launch: the whole GPU suite, cfg3 / cfg2 A/B
# against the 4-wave kernel, one SQ pass of the phi kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
source tools/fault_guard.sh
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_all.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/ab/pytest_all.log; fault_guard gpurun_out/ab/pytest_all.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="base SVGD_PHI_T8K=0" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
VARIANTS="base" BENCH_ARGS="--config cfg2" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
TAG=_r3b bash tools/pmc_sq.sh "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" || exit 1
