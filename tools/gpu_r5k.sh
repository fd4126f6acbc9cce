#!/bin/bash
# Round 5: the sharded symmetric phi pass -- its host-shm multi-rank tests,
# then the P = 8 / 4 shares (sim-world) with the row stream vs the symmetric
# pass over the rank's pair units (the reduce-scatter is not in a sim share).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r5k
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_multirank.py -k symmetric > $O/pytest.log 2>&1
rc=$?; fault_guard $O/pytest.log; tail -3 $O/pytest.log; [ $rc = 0 ] || exit 1
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); dg=d.get('diag_ms_per_step') or {}; h=d['host_ms_per_step']; print('$name', round(d['ms_per_step'],4), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']], 'phi', dg.get('phi_kernel'), 'phase', d.get('phase_ms_per_step'), 'grad', h.get('grad'), 'trk', d['tracked_brackets'])"
}
for i in 1 2; do :
  SVGD_PHI_SYM=0 b sim8_rows_$i 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
  SVGD_PHI_SYM=1 b sim8_sym_$i 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
  SVGD_PHI_SYM=0 b sim4_rows_$i 300 --sim-world 4 --steps 20 --warmup 5 --no-cpu
  SVGD_PHI_SYM=1 b sim4_sym_$i 300 --sim-world 4 --steps 20 --warmup 5 --no-cpu
done
echo r5k done
