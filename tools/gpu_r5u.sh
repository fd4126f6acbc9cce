#!/bin/bash
# Round 5: the cfg3 and cfg5 lines with the accuracy pre-pass moved after
# the timed runs (default arguments otherwise, CPU leg included).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r5u
mkdir -p $O
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); r=d['roofline']; cb=d.get('cpu_baseline') or {}; print('$name', round(d['ms_per_step'],4), d['value'], r.get('kernel_launched'), 'frac', r.get('frac'), 'traffic', r.get('traffic'), 'cpu', cb.get('value'), (cb.get('accuracy') or {}).get('phi_err_rel_to_max'), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']], 'clk', d['gpu_timed'].get('gfxclk_mhz_median'))"
}
b bench 600
b bench_cfg5 500 --config cfg5
echo r5u done
