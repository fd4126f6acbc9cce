#!/bin/bash
# Run-to-run stability of the headline bench (and cfg5 once).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/stab
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/stab/b$i.log 2>&1 || exit 1
  echo "cfg3 $i $(grep '^{' gpurun_out/stab/b$i.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), {k: round(v,3) for k,v in d["phases_ms_per_step"].items()})')"
done
timeout -k 10 300 python bench.py --config cfg5 --steps 20 --warmup 3 --no-cpu > gpurun_out/stab/c5.log 2>&1 || exit 1
echo "cfg5 $(grep '^{' gpurun_out/stab/c5.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), {k: round(v,3) for k,v in d["phases_ms_per_step"].items()})')"
