#!/bin/bash
# SQ counters of the cfg5 step's kernels (k_pair_tcol3, k_phi_b3): issue
# counts by type, MFMA busy, waits -- one pass per set.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=_r4q BENCH_ARGS="--config cfg5 --repeats 1 --no-diag" bash tools/pmc_sq.sh \
  "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_WAVES GRBM_GUI_ACTIVE" || exit 1
grep -h -i "coexec" gpurun_out/pmc_sq_r4q/avail.txt | head -3
echo r4q done
