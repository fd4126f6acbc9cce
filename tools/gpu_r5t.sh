#!/bin/bash
# Round 5: why the first timed runs of the default cfg3 line are slow (host
# gradient 5x slower) when the CPU leg is on: default, --no-cpu, and
# OMP_WAIT_POLICY=passive, alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r5t
mkdir -p $O
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); h=d['host_ms_per_step']; print('$name', round(d['ms_per_step'],4), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']], 'grad', round(h.get('grad'),3), 'job', round(h.get('job'),3), 'trk', d['tracked_brackets'])"
}
for i in 1 2; do
  b def_$i 600 --steps 20 --warmup 3 --cpu-rows 2048 --cpu-rows-1t 256
  b nocpu_$i 600 --steps 20 --warmup 3 --no-cpu
  OMP_WAIT_POLICY=passive b passive_$i 600 --steps 20 --warmup 3 --cpu-rows 2048 --cpu-rows-1t 256
done
echo r5t done
