#!/bin/bash
# Round 5: after the centring fold (one centring launch at every P) and the
# AVX-512-aware row-part policy -- the GPU suite, cfg3 / cfg2 lines, the
# 8-rank share (2x) with its kernel timeline, the 8-rank bench rehearsal.
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
source tools/fault_guard.sh
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -q tests \
  > $O/pytest_gpu.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -2 $O/pytest_gpu.log; fault_guard $O/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; }
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); dg=d.get('diag_ms_per_step') or {}; h=d['host_ms_per_step']; print('$name', round(d['ms_per_step'],4), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']], 'phi', dg.get('phi_kernel'), 'parts', dg.get('phi_launches_per_step'), 'wait', dg.get('phi_wait_for_g'), 'grad', h.get('grad'), 'trk', d['tracked_brackets'])"
}
b bench 600 --steps 20 --warmup 3 --no-cpu
b bench_cfg2 300 --config cfg2 --steps 20 --warmup 3 --no-cpu
b sim8_1 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
b sim8_2 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/$O/sim8 -o run --output-format csv \
   -- python3 $REPO/bench.py --sim-world 8 --steps 20 --warmup 3 --no-cpu > $REPO/$O/sim8_prof.log 2>&1) || exit 1
fault_guard $O/sim8_prof.log
python3 tools/step_timeline.py $O/sim8/run_kernel_trace.csv > $O/step_timeline_sim8.txt
cat $O/step_timeline_sim8.txt
CONFIGS="cfg2" bash tools/gpu_timeline.sh || exit 1
cp gpurun_out/timeline/cfg2.txt $O/step_timeline_cfg2.txt; cat $O/step_timeline_cfg2.txt
bash tools/rehearse_bench_mr.sh 8 $O/rehearsal_mr8.json || exit 1
echo r5c done
