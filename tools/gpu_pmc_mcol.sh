#!/bin/bash
# SQ counters of the collect pass (and the phi kernel) at cfg3 with tracked brackets
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
BENCH_ARGS="--steps 10 --warmup 10 --repeats 3" TAG=_mcol bash tools/pmc_sq.sh "SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" || exit 1
