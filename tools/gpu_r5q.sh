#!/bin/bash
# Round 5: X mirror A/B on the P = 4 share (sharded symmetric pass, 1 MiB
# shard: mirror on by default) and the P = 2 share (2 MiB: off by default).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r5q
mkdir -p $O
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); dg=d.get('diag_ms_per_step') or {}; print('$name', round(d['ms_per_step'],4), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']], 'phi', dg.get('phi_kernel'), 'wait', dg.get('phi_wait_for_g'), 'clk', d['gpu_timed'].get('gfxclk_mhz_median'))"
}
for i in 1 2; do
  SVGD_X_MIRROR=1 b sim4_m1_$i 300 --sim-world 4 --steps 20 --warmup 5 --no-cpu
  SVGD_X_MIRROR=0 b sim4_m0_$i 300 --sim-world 4 --steps 20 --warmup 5 --no-cpu
  SVGD_X_MIRROR=1 b sim2_m1_$i 300 --sim-world 2 --steps 20 --warmup 5 --no-cpu
  SVGD_X_MIRROR=0 b sim2_m0_$i 300 --sim-world 2 --steps 20 --warmup 5 --no-cpu
done
b p1_$i 300 --steps 20 --warmup 5 --no-cpu
echo r5q done
