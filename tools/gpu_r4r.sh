#!/bin/bash
# Round-4 final bench lines with the regenerated PMC roofline files (cfg3
# default with its CPU leg, cfg2, cfg5), plus smoke().
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4r
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "FAIL smoke"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); r=d['roofline']; cb=d.get('cpu_baseline') or {}; print('$name', round(d['ms_per_step'],4), d['value'], r.get('kernel_launched'), 'frac', r.get('frac'), 'traffic', r.get('traffic'), 'cpu', cb.get('value'), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']], 'clk', d['gpu_timed'].get('gfxclk_mhz_median'))"
}
b bench 600 --steps 20 --warmup 3
b bench_cfg2 400 --config cfg2 --steps 20 --warmup 3
b bench_cfg5 500 --config cfg5 --steps 20 --warmup 3
echo r4r done
