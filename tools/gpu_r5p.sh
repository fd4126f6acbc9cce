#!/bin/bash
# Round 5: SQ issue counters and L2 fetch of every kernel of the cfg3 step
# (the small kernels around the symmetric phi pass: finish, centring, record
# prep, median tail).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
TAG=_r5p BENCH_ARGS="--repeats 1 --no-diag" bash tools/pmc_sq.sh \
  "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
  "FETCH_SIZE SQ_WAVES SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE" || exit 1
python3 tools/pmc_summary.py gpurun_out/r5p_sq.csv gpurun_out/pmc_sq_r5p/p1 gpurun_out/pmc_sq_r5p/p2 || exit 1
cat gpurun_out/r5p_sq.csv | cut -c1-400
echo r5p done
