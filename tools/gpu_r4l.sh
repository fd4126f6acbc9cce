#!/bin/bash
# F32 collect classified on the bf16 matrix cores (k_pair_tcolb): the collect
# and F32 suites, same-box cfg5 lines against the fp32 classification
# (SVGD_TCOL_BF16=0), rocprof kernel means of the new default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_collect.py tests/test_gpu_f32.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest.log; fault_guard $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); dg=d.get('diag_ms_per_step') or {}; print('$name', round(d['ms_per_step'],4), 'phi', round(dg.get('phi_kernel'),4), 'phases', d['phases_ms_per_step'], 'clk', (d.get('gpu_diag') or {}).get('gfxclk_mhz_median'), 'path', d['median_path'])"
}
for i in 1 2; do
  SVGD_TCOL_BF16=0 b cfg5_tcol_$i 400 --config cfg5 --steps 20 --warmup 3 --no-cpu
  b cfg5_tcolb_$i 400 --config cfg5 --steps 20 --warmup 3 --no-cpu
done
STEPS=10 WARMUP=3 TAG=_tcolb BENCH_ARGS="--config cfg5 --repeats 1" bash tools/profile.sh > /dev/null || exit 1
python3 tools/ktimed.py gpurun_out/prof_tcolb/run_kernel_trace.csv 3 > $O/rocprof_cfg5_kernel_timed.txt
head -8 $O/rocprof_cfg5_kernel_timed.txt
echo r4l done
