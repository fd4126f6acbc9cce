#!/bin/bash
# cfg5 median phase vs the bracket width (SVGD_MEDIAN_SIGMA: the sampled
# bracket's sigmas; whole-tile samples take 4x), two interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4o
mkdir -p $O
for i in 1 2; do
  for s in 3 2 1.5 1; do
    SVGD_MEDIAN_SIGMA=$s timeout -k 10 300 python bench.py --config cfg5 --steps 20 --warmup 3 --no-cpu --repeats 3 > $O/s$s.$i.log 2>&1 || { echo "FAIL $s"; tail -5 $O/s$s.$i.log; exit 1; }
    fault_guard $O/s$s.$i.log
    tail -1 $O/s$s.$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('sigma $s', $i, round(d['ms_per_step'],4), 'med', round(d['phases_ms_per_step']['median_incl_step_gap'],4), 'trk', d.get('tracked_brackets'), 'clk', d['gpu_timed'].get('gfxclk_mhz_median'))"
  done
done
echo r4o done
