#!/bin/bash
# F32 median keys on the bf16 matrix cores (KP 32 / 64) and the mean
# partials from the update epilogue: the whole GPU suite, then cfg5 / cfg2 /
# cfg3 lines and a rocprof pass of cfg5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest.log; fault_guard $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); dg=d.get('diag_ms_per_step') or {}; print('$name', round(d['ms_per_step'],4), 'phi', round(dg.get('phi_kernel') or 0,4), 'phases', {k: round(v,4) for k,v in (d.get('phases_ms_per_step') or {}).items()}, 'clk', (d.get('gpu_diag') or {}).get('gfxclk_mhz_median'))"
}
for i in 1 2; do
  b cfg5.$i 300 --config cfg5 --steps 20 --warmup 3 --no-cpu
  b cfg2.$i 300 --config cfg2 --steps 20 --warmup 3 --no-cpu
done
b cfg3 300 --steps 20 --warmup 3 --no-cpu
STEPS=10 WARMUP=3 TAG=_r4m BENCH_ARGS="--config cfg5 --repeats 1" bash tools/profile.sh > /dev/null || exit 1
python3 tools/ktimed.py gpurun_out/prof_r4m/run_kernel_trace.csv 3 > $O/rocprof_cfg5_kernel_timed.txt
head -6 $O/rocprof_cfg5_kernel_timed.txt
CONFIGS="cfg2" bash tools/gpu_timeline.sh || exit 1
cp gpurun_out/timeline/cfg2.txt $O/step_timeline_cfg2.txt
cat $O/step_timeline_cfg2.txt
echo r4m done
