#!/bin/bash
# Round 5: cfg4 (N = 262144) 8-rank share, row stream (default at P = 8) vs
# the sharded symmetric pass, same box alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r5y
mkdir -p $O
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); dg=d.get('diag_ms_per_step') or {}; print('$name', round(d['ms_per_step'],4), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']], 'phi', dg.get('phi_kernel'), 'parts', dg.get('phi_launches_per_step'), 'clk', d['gpu_timed'].get('gfxclk_mhz_median'))"
}
for i in 1 2; do
  SVGD_PHI_SYM=0 b cfg4_sim8_rows_$i 400 --config cfg4 --sim-world 8 --steps 10 --warmup 3 --repeats 3 --no-cpu
  SVGD_PHI_SYM=1 b cfg4_sim8_sym_$i 400 --config cfg4 --sim-world 8 --steps 10 --warmup 3 --repeats 3 --no-cpu
done
echo r5y done
