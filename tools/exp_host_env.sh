#!/bin/bash
# Headline bench under host-threading variants (same box, alternating).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/hostenv
echo "nproc $(nproc) affinity $(taskset -pc $$ 2>/dev/null | sed 's/.*: //') OMP_NUM_THREADS=$OMP_NUM_THREADS"
for i in 1 2 3; do
  for mode in default passive t8; do
    case $mode in
      default) env="" ;;
      passive) env="OMP_WAIT_POLICY=PASSIVE" ;;
      t8) env="OMP_NUM_THREADS=8" ;;
    esac
    env $env timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/hostenv/$mode$i.log 2>&1 || exit 1
    echo "$mode $i $(grep '^{' gpurun_out/hostenv/$mode$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), {k: round(v,3) for k,v in d["phases_ms_per_step"].items()})')"
  done
done
