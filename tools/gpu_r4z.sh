#!/bin/bash
# cfg5 and cfg4 under the N-dependent tracked-bracket width (2.5) vs the old 4, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4z
mkdir -p $O
for i in 1 2; do
  for v in X=1 SVGD_TRACK_ERR_MULT=4; do
    env $v timeout -k 10 300 python bench.py --config cfg5 --steps 30 --warmup 3 --no-cpu --repeats 3 --no-diag > $O/cfg5_$v.$i.log 2>&1 || { echo "FAIL $v"; tail -3 $O/cfg5_$v.$i.log; exit 1; }
    fault_guard $O/cfg5_$v.$i.log
    tail -1 $O/cfg5_$v.$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg5 $v', $i, round(d['ms_per_step'],4), 'runs', [round(x,4) for x in d['repeats']['ms_per_step']], 'med', round(d['phases_ms_per_step']['median_incl_step_gap'],4), 'trk', d['tracked_brackets'], 'clk', d['gpu_timed'].get('gfxclk_mhz_median'))"
  done
done
echo r4z done
