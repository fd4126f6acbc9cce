#!/bin/bash
# Round-5 evidence, part 2 (final sources): the whole GPU suite, smoke(), a
# bench line for every BASELINE config (CPU legs), the C++ SVGD::Run line,
# and full-size multi-rank bench rehearsals (host-shm) at 2, 4, 8 ranks and
# 8 ranks with the sharded symmetric pass forced.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r5f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; fault_guard $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" $O/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
fault_guard $O/smoke.log; tail -1 $O/smoke.log
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); r=d['roofline']; cb=d.get('cpu_baseline') or {}; print('$name', round(d['ms_per_step'],4), round(d['value']/1e6,3), r.get('kernel_launched'), 'frac', round(r.get('frac') or 0,3), 'traffic', r.get('traffic'), 'cpu', cb.get('value'), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']], 'clk', d['gpu_timed'].get('gfxclk_mhz_median'))"
}
b bench 600
b bench_cfg2 400 --config cfg2
b bench_cfg5 500 --config cfg5
b bench_cfg4 900 --config cfg4 --steps 5 --warmup 2 --repeats 3
b bench_cfg5_f64 400 --config cfg5 --dtype f64 --steps 5 --warmup 2 --repeats 3 --no-cpu
(cd build && timeout -k 10 300 ./svgd_run_bench > ../$O/bench_cpp.log 2>&1) || { tail -5 $O/bench_cpp.log; exit 1; }
fault_guard $O/bench_cpp.log
grep '^{' $O/bench_cpp.log | tail -1 > $O/bench_cpp.json; python3 -c "import json; d=json.load(open('$O/bench_cpp.json')); print('cpp', d['ms_per_step'], d['repeats']['ms_per_step'])"
for N in 2 4 8; do
  bash tools/rehearse_bench_mr.sh $N $O/rehearsal_mr$N.json || exit 1
  fault_guard gpurun_out/bench_mr$N.log
done
SVGD_PHI_SYM=1 bash tools/rehearse_bench_mr.sh 8 $O/rehearsal_mr8_sym.json || exit 1
fault_guard gpurun_out/bench_mr8.log
echo r5final done
