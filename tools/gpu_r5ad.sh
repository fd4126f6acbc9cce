#!/bin/bash
# Round 5: the 8-rank cfg3 share with the rank's gradient threads at the
# 16-CPU box's share (2) vs 4 and 8 (a node with more CPUs per GPU), row
# stream and symmetric pass -- how much of the share's fixed cost is the
# host gradient's hand-over.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r5ad
mkdir -p $O
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); dg=d.get('diag_ms_per_step') or {}; h=d['host_ms_per_step']; print('$name', round(d['ms_per_step'],4), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']], 'phi', round(dg.get('phi_kernel') or 0,4), 'wait', round(dg.get('phi_wait_for_g') or 0,4), 'grad', round(h.get('grad'),4), 'thr', h.get('threads'))"
}
for i in 1 2; do
  for t in 2 4 8; do
    SVGD_HOST_THREADS=$t b t${t}_$i 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
  done
  SVGD_HOST_THREADS=8 SVGD_PHI_SYM=1 b t8sym_$i 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
done
echo r5ad done
