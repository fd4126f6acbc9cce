#!/bin/bash
# Round 4, second call: the median/step suites touched by the adaptive
# speculative cap and the row-half phi, then cfg4 (one GPU) and the per-rank
# shares with the quota/P gradient threads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_model_step.py tests/test_gpu_multirank.py tests/test_gpu_speculative.py tests/test_gpu_track.py tests/test_gpu_median_paths.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest.log; fault_guard $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" $O/pytest.log | head; exit $rc; }
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); r=d['roofline']; dg=d.get('diag_ms_per_step') or {}; print('$name', round(d['ms_per_step'],4), 'frac', r.get('frac'), 'phi', dg.get('phi_kernel'), 'parts', dg.get('phi_launches_per_step'), 'wait', dg.get('phi_wait_for_g'), 'thr', d['host_ms_per_step'].get('threads'), 'trk', d['tracked_brackets'])"
}
b sim8_cfg3 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
SVGD_PHI_SPLIT=0 b sim8_cfg3_nosplit 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
b sim4_cfg3 300 --sim-world 4 --steps 20 --warmup 5 --no-cpu
b sim2_cfg3 300 --sim-world 2 --steps 20 --warmup 5 --no-cpu
b sim8_cfg4 400 --config cfg4 --sim-world 8 --steps 10 --warmup 3 --no-cpu
b cfg4 900 --config cfg4 --steps 5 --warmup 3 --repeats 3 --no-cpu
b cfg3 600 --steps 20 --warmup 3 --no-cpu
echo r4b done
