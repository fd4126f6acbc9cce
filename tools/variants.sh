#!/bin/bash
# A/B timing of kernel variants selected by environment variables (one bench
# line each, no CPU leg).  Usage: bash tools/variants.sh "ENV=.. ENV2=.." ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/variants
source tools/fault_guard.sh
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu ${BENCH_ARGS:-} > gpurun_out/variants/v$i.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/variants/v$i.log; exit 1; }
  fault_guard gpurun_out/variants/v$i.log
  tail -1 gpurun_out/variants/v$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step'],3), {k: round(x,3) for k,x in d['phases_ms_per_step'].items()})"
done
