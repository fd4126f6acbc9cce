#!/bin/bash
# F32 tile phi on the bf16 matrix cores (k_phi_b3, SVGD_PHI_B3=1): the F32
# suite with it on, then same-box cfg5 lines and rocprof means, B3 vs f32s.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_f32.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest.log; fault_guard $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
SVGD_PHI_B3=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_f32.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_b3.log 2>&1; rc=$?
echo "pytest b3 rc=$rc"; tail -1 $O/pytest_b3.log; fault_guard $O/pytest_b3.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest_b3.log | head -20; exit $rc; }
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); r=d['roofline']; dg=d.get('diag_ms_per_step') or {}; print('$name', round(d['ms_per_step'],4), r.get('kernel_launched'), 'frac', r.get('frac'), 'phi', dg.get('phi_kernel'), 'clk', (d.get('gpu_diag') or {}).get('gfxclk_mhz_median'), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']])"
}
for i in 1 2; do
  SVGD_PHI_B3=0 b cfg5_f32s_$i 400 --config cfg5 --steps 20 --warmup 3 --no-cpu
  b cfg5_b3_$i 400 --config cfg5 --steps 20 --warmup 3 --no-cpu
done
unset SVGD_PHI_B3
STEPS=10 WARMUP=3 TAG=_b3 BENCH_ARGS="--config cfg5 --repeats 1" bash tools/profile.sh > /dev/null || exit 1
python3 tools/ktimed.py gpurun_out/prof_b3/run_kernel_trace.csv 3 > $O/rocprof_cfg5_b3_kernel_timed.txt
head -6 $O/rocprof_cfg5_b3_kernel_timed.txt
TAG=_b3 BENCH_ARGS="--config cfg5 --repeats 1 --no-diag" bash tools/pmc_sq.sh "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE" || exit 1
python3 tools/pmc_summary.py $O/pmc_sq_b3.csv gpurun_out/pmc_sq_b3/p1 > $O/pmc_sq_b3.txt
python3 tools/pmc_summary.py $O/pmc_lds_b3.csv gpurun_out/pmc_sq_b3/p2 > $O/pmc_lds_b3.txt
head -1 $O/pmc_sq_b3.txt | cut -c1-600; head -1 $O/pmc_lds_b3.txt | cut -c1-600
echo r4j done
