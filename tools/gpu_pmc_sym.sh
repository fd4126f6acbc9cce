#!/bin/bash
# SQ counters of the phi kernels: row stream (base) vs the symmetric pass, cfg3 and cfg2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
A="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
B="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F64 SQ_WAIT_ANY SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
for cfg in cfg3 cfg2; do
  for v in base sym; do
    if [ $v = sym ]; then export SVGD_PHI_SYM=1; else unset SVGD_PHI_SYM; fi
    TAG=_${cfg}_$v BENCH_ARGS="--config $cfg --no-diag --repeats 1" bash tools/pmc_sq.sh "$A" "$B" || exit 1
    python3 tools/pmc_summary.py gpurun_out/pmc_sq_${cfg}_$v/summary.csv gpurun_out/pmc_sq_${cfg}_$v/p1 gpurun_out/pmc_sq_${cfg}_$v/p2
  done
done
unset SVGD_PHI_SYM
echo done
