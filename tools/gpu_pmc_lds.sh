#!/bin/bash
# LDS behaviour of the phi row stream (bank conflicts of the random exp-table
# reads, LDS waits): one counter pass at cfg3, plus the RCCL tracked test
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_rccl.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab/pytest_rccl.log; [ $rc -ne 0 ] && exit $rc
TAG=_lds bash tools/pmc_sq.sh "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE" || exit 1
