#!/bin/bash
# First-run slowness on a fresh box: long warm-up first, then the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/warm
for w in 200 3 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup $w --no-cpu > gpurun_out/warm/w$w.log 2>&1 || exit 1
  echo "warmup $w $(grep '^{' gpurun_out/warm/w$w.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), {k: round(v,3) for k,v in d["phases_ms_per_step"].items()})')"
done
