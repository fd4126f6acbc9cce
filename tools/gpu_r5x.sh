#!/bin/bash
# Round 5: SQ counters of k_phi_sym<2> at cfg2 (why it ties the row stream there).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
SVGD_PHI_SYM=1 TAG=_cfg2sym BENCH_ARGS="--config cfg2 --repeats 1 --no-diag" bash tools/pmc_sq.sh \
  "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" || exit 1
python3 tools/pmc_summary.py gpurun_out/r5x_sq.csv gpurun_out/pmc_sq_cfg2sym/p1 gpurun_out/pmc_sq_cfg2sym/p2 || exit 1
grep -E "k_phi_sym|k_phi_rows|kernel," gpurun_out/r5x_sq.csv | cut -c1-600
echo r5x done
