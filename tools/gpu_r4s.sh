#!/bin/bash
# cfg2 fixed costs: host gradient threads (SVGD_HOST_THREADS) and the G
# host read (SVGD_G_HOSTREAD), interleaved, with the phi wait for G.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4s
mkdir -p $O
for i in 1 2; do
  for v in base SVGD_HOST_THREADS=1 SVGD_HOST_THREADS=2 SVGD_HOST_THREADS=4 SVGD_G_HOSTREAD=0; do
    if [ "$v" = base ]; then envs=""; else envs="$v"; fi
    env $envs timeout -k 10 300 python bench.py --config cfg2 --steps 40 --warmup 5 --no-cpu --repeats 3 > $O/$v.$i.log 2>&1 || { echo "FAIL $v"; tail -3 $O/$v.$i.log; exit 1; }
    fault_guard $O/$v.$i.log
    tail -1 $O/$v.$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); h=d['host_ms_per_step']; dg=d['diag_ms_per_step']; print('$v', $i, round(d['ms_per_step'],4), 'runs', [round(x,4) for x in d['repeats']['ms_per_step']], 'grad', round(h['grad'],4), 'xwait', round(h['xwait'],4), 'wait_g', round(dg.get('phi_wait_for_g') or 0,4), 'clk', d['gpu_timed'].get('gfxclk_mhz_median'))"
  done
done
echo r4s done
