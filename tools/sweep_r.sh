#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2 4; do
  SVGD_PHI_R=$r timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_r$r.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_r$r.log').read().strip().splitlines()[-1]); print('R=$r', round(d['ms_per_step'],3), d['phases_ms_per_step'], round(d['roofline']['frac'],3))"
done
