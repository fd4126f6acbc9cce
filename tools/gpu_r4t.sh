#!/bin/bash
# cfg2 with the G copies by default: host-model step tests, cfg2 lines (two
# rounds), its step timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4t
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_host_model_step.py tests/test_gpu_speculative.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest.log; fault_guard $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --config cfg2 --steps 40 --warmup 5 --no-cpu --repeats 5 > $O/cfg2.$i.log 2>&1 || { echo FAIL; tail -3 $O/cfg2.$i.log; exit 1; }
  fault_guard $O/cfg2.$i.log
  tail -1 $O/cfg2.$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); dg=d['diag_ms_per_step']; print('cfg2', $i, round(d['ms_per_step'],4), 'runs', [round(x,4) for x in d['repeats']['ms_per_step']], 'wait_g', round(dg.get('phi_wait_for_g') or 0,4), 'clk', d['gpu_timed'].get('gfxclk_mhz_median'))"
done
CONFIGS="cfg2" bash tools/gpu_timeline.sh || exit 1
cp gpurun_out/timeline/cfg2.txt $O/step_timeline_cfg2.txt; cat $O/step_timeline_cfg2.txt
echo r4t done
