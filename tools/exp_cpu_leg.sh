#!/bin/bash
# Headline bench with and without the CPU-baseline leg, alternating (same box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cpuleg
for i in 1 2; do
  for mode in nocpu cpu; do
    args=""; [ $mode = nocpu ] && args="--no-cpu"
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 $args > gpurun_out/cpuleg/$mode$i.log 2>&1 || exit 1
    echo "$mode $i $(tail -1 gpurun_out/cpuleg/$mode$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), {k: round(v,3) for k,v in d["phases_ms_per_step"].items()})')"
  done
done
