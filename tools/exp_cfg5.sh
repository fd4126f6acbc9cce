#!/bin/bash
# cfg5 experiment: host-gradient timing (C++ driver) and bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cfg5
test -x build/host_grad_bench || exit 1
for t in 1 16; do OMP_NUM_THREADS=$t timeout -k 10 60 build/host_grad_bench | tail -1 | sed "s/^/host grad threads=$t: /"; done
for i in 1 2; do
  timeout -k 10 120 python bench.py --config cfg5 --steps 20 --warmup 3 --no-cpu > gpurun_out/cfg5/b$i.log 2>&1 || exit 1
  tail -1 gpurun_out/cfg5/b$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["phases_ms_per_step"])'
done
