#!/bin/bash
# Round 5: the host gradient builds on the box's CPU (AVX2 block vs the
# AVX-512 structure-of-arrays block, bit-identical results) and the 8-rank
# share with and without the two phi row parts (sim-world, quota/P threads).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r5b
mkdir -p $O
for a in "8192 8 4 2" "8192 8 4 1" "65536 8 4 8" "65536 64 1 16" "65536 64 1 1" "16384 2 1 8"; do
  timeout -k 5 120 ./build/host_grad_bench $a || exit 1
done | tee $O/host_grad.txt
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); dg=d.get('diag_ms_per_step') or {}; h=d['host_ms_per_step']; print('$name', round(d['ms_per_step'],4), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']], 'phi', dg.get('phi_kernel'), 'parts', dg.get('phi_launches_per_step'), 'wait', dg.get('phi_wait_for_g'), 'grad', h.get('grad'), 'thr', h.get('threads'), 'trk', d['tracked_brackets'])"
}
for i in 1 2; do
  SVGD_PHI_SPLIT=1 b sim8_split_$i 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
  SVGD_PHI_SPLIT=0 b sim8_whole_$i 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
  SVGD_PHI_SPLIT=1 b sim4_split_$i 300 --sim-world 4 --steps 20 --warmup 5 --no-cpu
  SVGD_PHI_SPLIT=0 b sim4_whole_$i 300 --sim-world 4 --steps 20 --warmup 5 --no-cpu
done
echo r5b done
