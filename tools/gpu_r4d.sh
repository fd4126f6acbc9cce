#!/bin/bash
# Round 4: (1) the rebuilt symmetric phi pass (r4c's suite: parity, same-box
# A/B against the row stream, rocprof, SQ counters); (2) the fp64 tile phi
# (8-wave blocks, j-major LDS, VALU row sums): parity and a same-box A/B of
# library builds at N = 65536, d = 64 fp64.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_sym.py tests/test_gpu_parity.py tests/test_gpu_host_model_step.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest.log; fault_guard $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); r=d['roofline']; dg=d.get('diag_ms_per_step') or {}; print('$name', round(d['ms_per_step'],4), r.get('kernel_launched'), 'frac', r.get('frac'), 'phi', dg.get('phi_kernel'), 'wait', dg.get('phi_wait_for_g'), 'clk', (d.get('gpu_diag') or {}).get('gfxclk_mhz_median'), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']])"
}
# fp64 d = 64 tile phi: library builds on one box
LIB=svgdcpp_amd/libsvgdcpp_amd.so
cp $LIB $O/.cur.so
for v in base p1w1 p0w4 p0w1 base p1w1 p0w4; do
  cp tools/ablibs/$v.so $LIB
  b t64_$v 300 --config cfg5 --dtype f64 --steps 5 --warmup 2 --repeats 3 --no-cpu || { cp $O/.cur.so $LIB; exit 1; }
done
cp $O/.cur.so $LIB
SVGD_PHI_S1V=0 b t64_cur_nos1v 300 --config cfg5 --dtype f64 --steps 5 --warmup 2 --repeats 3 --no-cpu
for i in 1 2; do
  SVGD_X_MIRROR=0 SVGD_G_HOSTREAD=0 b cfg2_copy_$i 300 --config cfg2 --steps 20 --warmup 3 --no-cpu
  b cfg2_zc_$i 300 --config cfg2 --steps 20 --warmup 3 --no-cpu
done
SVGD_X_MIRROR=0 b sim8_copy 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
for f in 50 62 72; do
  SVGD_PHI_SPLIT_FRAC=$f b sim8_f$f 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
done
SVGD_PHI_SPLIT_FRAC=62 b sim4_f62 300 --sim-world 4 --steps 20 --warmup 5 --no-cpu
for i in 1 2; do
  SVGD_PHI_SYM=0 b rows_cfg3_$i 300 --steps 20 --warmup 3 --no-cpu
  SVGD_PHI_SYM=1 b sym_cfg3_$i 300 --steps 20 --warmup 3 --no-cpu
done
SVGD_PHI_SYM=0 b rows_cfg2 300 --config cfg2 --steps 20 --warmup 3 --no-cpu
SVGD_PHI_SYM=1 b sym_cfg2 300 --config cfg2 --steps 20 --warmup 3 --no-cpu
export SVGD_PHI_SYM=1
STEPS=20 WARMUP=3 TAG=_sym bash tools/profile.sh > /dev/null || exit 1
python3 tools/ktimed.py gpurun_out/prof_sym/run_kernel_trace.csv 3 > $O/rocprof_sym_kernel_timed.txt
head -6 $O/rocprof_sym_kernel_timed.txt
TAG=_sym BENCH_ARGS="--repeats 1 --no-diag" bash tools/pmc_sq.sh "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE" || exit 1
python3 tools/pmc_summary.py $O/pmc_sq_sym.csv gpurun_out/pmc_sq_sym/p1 > $O/pmc_sq_sym.txt
python3 tools/pmc_summary.py $O/pmc_lds_sym.csv gpurun_out/pmc_sq_sym/p2 > $O/pmc_lds_sym.txt
head -3 $O/pmc_sq_sym.txt
echo r4d done
