#!/bin/bash
# Round 5: cfg5 sampled-bracket width -- sample size and sigma variants
# (same box, alternated), median paths and misses in each line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r5ab
mkdir -p $O
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); print('$name', round(d['ms_per_step'],4), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']], 'phases', {k: round(v,3) for k,v in d['phases_ms_per_step'].items()}, 'trk', d['tracked_brackets'], 'path', d.get('median_path'))"
}
for i in 1 2; do
  b base_$i 400 --config cfg5 --no-cpu --no-diag
  SVGD_MEDIAN_SIGMA=2 b sig2_$i 400 --config cfg5 --no-cpu --no-diag
  SVGD_MEDIAN_SAMPLE=16777216 b s24_$i 400 --config cfg5 --no-cpu --no-diag
  SVGD_MEDIAN_SAMPLE=16777216 SVGD_MEDIAN_SIGMA=1.5 b s24sig15_$i 400 --config cfg5 --no-cpu --no-diag
done
echo r5ab done
