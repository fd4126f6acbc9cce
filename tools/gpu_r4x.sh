#!/bin/bash
# cfg3 tracked-bracket width (SVGD_TRACK_ERR_MULT: half-width / recent
# prediction error, default 4), three interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4x
mkdir -p $O
for i in 1 2 3; do
  for v in base SVGD_TRACK_ERR_MULT=3 SVGD_TRACK_ERR_MULT=2.5; do
    if [ "$v" = base ]; then envs=""; else envs="$v"; fi
    env $envs timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --repeats 3 --no-diag > $O/$v.$i.log 2>&1 || { echo "FAIL $v"; tail -3 $O/$v.$i.log; exit 1; }
    fault_guard $O/$v.$i.log
    tail -1 $O/$v.$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', $i, round(d['ms_per_step'],4), 'runs', [round(x,4) for x in d['repeats']['ms_per_step']], 'med', round(d['phases_ms_per_step']['median_incl_step_gap'],4), 'trk', d['tracked_brackets'], 'clk', d['gpu_timed'].get('gfxclk_mhz_median'))"
  done
done
echo r4x done
