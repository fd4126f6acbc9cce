#!/bin/bash
# Events between a step's kernels with a device-scope release
# (SVGD_EV_SCOPE=device) vs the default system scope: the step suites with
# it on, then interleaved same-box lines (cfg2, cfg3, 8-rank share).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4i
mkdir -p $O
SVGD_EV_SCOPE=device timeout -k 10 600 python -u -m pytest tests/test_gpu_host_model_step.py tests/test_gpu_multirank.py tests/test_gpu_speculative.py tests/test_gpu_track.py tests/test_gpu_parity.py tests/test_gpu_collect.py tests/test_gpu_median_paths.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest.log; fault_guard $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" $O/pytest.log | head; exit $rc; }
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); dg=d.get('diag_ms_per_step') or {}; print('$name', round(d['ms_per_step'],4), 'phi', round(dg.get('phi_kernel'),4), 'clk', (d.get('gpu_diag') or {}).get('gfxclk_mhz_median'), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']])"
}
for i in 1 2; do
  b cfg2_sys_$i 300 --config cfg2 --steps 20 --warmup 3 --no-cpu
  SVGD_EV_SCOPE=device b cfg2_dev_$i 300 --config cfg2 --steps 20 --warmup 3 --no-cpu
done
for i in 1 2; do
  b cfg3_sys_$i 300 --steps 20 --warmup 3 --no-cpu
  SVGD_EV_SCOPE=device b cfg3_dev_$i 300 --steps 20 --warmup 3 --no-cpu
done
b sim8_sys 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
SVGD_EV_SCOPE=device b sim8_dev 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
b f64_d64 400 --config cfg5 --dtype f64 --steps 5 --warmup 2 --repeats 3 --no-cpu
python3 -c "import json; d=json.load(open('$O/f64_d64.json')); print('f64 phases', d['phases_ms_per_step'])"
echo r4i done
