#!/bin/bash
# Round 5: the one-rank RCCL reduce-scatter of the sharded symmetric form,
# then the P = 2 / 4 / 8 shares (sim-world, cfg3) row stream vs symmetric,
# and the P = 1 cfg3 step timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r5m
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_rccl.py > $O/pytest.log 2>&1
rc=$?; fault_guard $O/pytest.log; tail -3 $O/pytest.log; [ $rc = 0 ] || exit 1
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); dg=d.get('diag_ms_per_step') or {}; print('$name', round(d['ms_per_step'],4), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']], 'phi', dg.get('phi_kernel'), 'clk', d['gpu_timed'].get('gfxclk_mhz_median'))"
}
for i in 1 2; do
  for P in 8 4 2; do
    SVGD_PHI_SYM=0 b sim${P}_rows_$i 300 --sim-world $P --steps 20 --warmup 5 --no-cpu
    SVGD_PHI_SYM=1 b sim${P}_sym_$i 300 --sim-world $P --steps 20 --warmup 5 --no-cpu
  done
done
CONFIGS="cfg3" bash tools/gpu_timeline.sh || exit 1
cat gpurun_out/timeline/cfg3.txt
echo r5m done
