#!/bin/bash
# A/B timing of environment settings on one box: each variant "name:VAR=v[,VAR=v]"
# runs one bench line per round (ROUNDS interleaved passes), BENCH_ARGS added.
# Usage: ROUNDS=2 BENCH_ARGS="--sim-world 8" bash tools/ab_env.sh on:SVGD_X_MIRROR=1 off:SVGD_X_MIRROR=0
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
source tools/fault_guard.sh
for round in $(seq ${ROUNDS:-2}); do
  for spec in "$@"; do
    name=${spec%%:*}; envs=${spec#*:}
    log=gpurun_out/ab/${TAG:-}$name.$round.log
    env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 3 --no-cpu ${BENCH_ARGS:-} > $log 2>&1 \
      || { echo "$name failed"; tail -5 $log; exit 1; }
    fault_guard $log
    tail -1 $log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('per_rank',[{}])[0] if d.get('per_rank') else d; print('$name', round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['phases_ms_per_step'].items() if isinstance(x, float)}, {k: round(x,4) for k,x in (d.get('diag_ms_per_step') or {}).items() if isinstance(x, float)})"
  done
done
