#!/bin/bash
# Round 5: SQ / LDS counters of the symmetric phi pass and the collect at cfg3.
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
source tools/fault_guard.sh
TAG=_r5j BENCH_ARGS="--repeats 1 --no-diag" bash tools/pmc_sq.sh "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" || exit 1
python3 tools/pmc_summary.py gpurun_out/r5j_sq.csv gpurun_out/pmc_sq_r5j/p1 || exit 1
python3 tools/pmc_summary.py gpurun_out/r5j_lds.csv gpurun_out/pmc_sq_r5j/p2 || exit 1
head -4 gpurun_out/r5j_sq.csv; head -4 gpurun_out/r5j_lds.csv
echo r5j done
