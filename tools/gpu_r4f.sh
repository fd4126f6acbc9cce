#!/bin/bash
# Symmetric phi with the 4 groups on one column set per phase (record reads
# broadcast 4 ways): parity suite, same-box A/B against the row stream at
# cfg3 (x2) and cfg2, SQ + LDS counters of k_phi_sym.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_sym.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_sym.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest_sym.log; fault_guard $O/pytest_sym.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest_sym.log | head -20; exit $rc; }
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); r=d['roofline']; dg=d.get('diag_ms_per_step') or {}; print('$name', round(d['ms_per_step'],4), r.get('kernel_launched'), 'phi', dg.get('phi_kernel'), 'clk', (d.get('gpu_diag') or {}).get('gfxclk_mhz_median'), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']])"
}
for i in 1 2; do
  SVGD_PHI_SYM=0 b rows_cfg3_$i 300 --steps 20 --warmup 3 --no-cpu
  SVGD_PHI_SYM=1 b sym_cfg3_$i 300 --steps 20 --warmup 3 --no-cpu
done
SVGD_PHI_SYM=1 b sym_cfg2 300 --config cfg2 --steps 20 --warmup 3 --no-cpu
export SVGD_PHI_SYM=1
TAG=_sym2 BENCH_ARGS="--repeats 1 --no-diag" bash tools/pmc_sq.sh "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE" || exit 1
python3 tools/pmc_summary.py $O/pmc_sq_sym.csv gpurun_out/pmc_sq_sym2/p1 > $O/pmc_sq_sym.txt
python3 tools/pmc_summary.py $O/pmc_lds_sym.csv gpurun_out/pmc_sq_sym2/p2 > $O/pmc_lds_sym.txt
head -1 $O/pmc_sq_sym.txt | cut -c1-400; head -1 $O/pmc_lds_sym.txt | cut -c1-500
echo r4f done
