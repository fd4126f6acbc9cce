#!/bin/bash
# Round evidence, part 2 (R=<round tag>): the whole GPU suite, smoke(), then
# a bench line for every BASELINE config on one GPU (cfg3 default with the
# CPU leg; cfg2, cfg5 and cfg4 full size with theirs; fp64 d = 64 without)
# and the C++ SVGD::Run line at cfg3.  SKIP_PYTEST=1 skips the suite.
#   R=r06 bash tools/evidence_suite.sh  -> gpurun_out/<R>r/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
R=${R:-rXX}
O=gpurun_out/${R}r
mkdir -p $O
if [ -z "$SKIP_PYTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; fault_guard $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" $O/pytest_gpu.log | head; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
  fault_guard $O/smoke.log; tail -2 $O/smoke.log
fi
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); r=d['roofline']; cb=d.get('cpu_baseline') or {}; print('$name', round(d['ms_per_step'],4), d['value'], r.get('kernel_launched'), 'frac', r.get('frac'), 'traffic', r.get('traffic'), 'cpu', cb.get('value'), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']])"
}
for cfg in ${CONFIGS:-cfg3 cfg2 cfg5 cfg4 cfg5_f64}; do
  case $cfg in
    cfg3) b bench 600 --steps 20 --warmup 3 ;;
    cfg2) b bench_cfg2 400 --config cfg2 --steps 20 --warmup 3 ;;
    cfg5) b bench_cfg5 500 --config cfg5 --steps 20 --warmup 3 ;;
    cfg4) b bench_cfg4 900 --config cfg4 --steps 5 --warmup 2 --repeats 3 ;;
    cfg5_f64) b bench_cfg5_f64 400 --config cfg5 --dtype f64 --steps 5 --warmup 2 --repeats 3 --no-cpu ;;
  esac
done
if [ -z "$SKIP_CPP" ]; then
  (cd build && timeout -k 10 300 ./svgd_run_bench > ../$O/bench_cpp.log 2>&1) || { tail -5 $O/bench_cpp.log; exit 1; }
  fault_guard $O/bench_cpp.log
  grep '^{' $O/bench_cpp.log | tail -1 > $O/bench_cpp.json; cut -c1-300 $O/bench_cpp.json
fi
echo "evidence_suite $R done"
