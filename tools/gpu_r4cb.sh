#!/bin/bash
# cfg5 collect grid (SVGD_COLLECT_BLOCKS; k_pair_tcol3 holds 2 blocks per CU), two interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4cb
mkdir -p $O
for i in 1 2; do
  for v in X=1 SVGD_COLLECT_BLOCKS=512 SVGD_COLLECT_BLOCKS=768 SVGD_COLLECT_BLOCKS=2048; do
    env $v timeout -k 10 300 python bench.py --config cfg5 --steps 20 --warmup 3 --no-cpu --repeats 3 > $O/$v.$i.log 2>&1 || { echo "FAIL $v"; tail -3 $O/$v.$i.log; exit 1; }
    fault_guard $O/$v.$i.log
    tail -1 $O/$v.$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', $i, round(d['ms_per_step'],4), 'med', round(d['phases_ms_per_step']['median_incl_step_gap'],4), 'clk', d['gpu_timed'].get('gfxclk_mhz_median'))"
  done
done
echo r4cb done
