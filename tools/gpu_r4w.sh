#!/bin/bash
# k_center_t (tile-path centring, fused fp32 copies): parity + F32 + collect
# suites, cfg5 / fp64 d=64 lines and a cfg5 rocprof pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_f32.py tests/test_gpu_collect.py tests/test_gpu_median_paths.py tests/test_gpu_matrix_scale.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest.log; fault_guard $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for a in "cfg5" "cfg5 --dtype f64"; do
  n=${a// /_}
  timeout -k 10 300 python bench.py --config $a --steps 10 --warmup 3 --no-cpu --repeats 3 > $O/$n.log 2>&1 || { echo FAIL $n; tail -3 $O/$n.log; exit 1; }
  fault_guard $O/$n.log
  tail -1 $O/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['ms_per_step'],4), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']], 'med', round(d['phases_ms_per_step']['median_incl_step_gap'],4), 'clk', d['gpu_timed'].get('gfxclk_mhz_median'))"
done
STEPS=10 WARMUP=3 TAG=_r4w BENCH_ARGS="--config cfg5 --repeats 1" bash tools/profile.sh > /dev/null || exit 1
python3 tools/ktimed.py gpurun_out/prof_r4w/run_kernel_trace.csv 3 > $O/rocprof_cfg5_kernel_timed.txt
grep -E "k_center|k_cvt|k_mean|k_swz" $O/rocprof_cfg5_kernel_timed.txt
echo r4w done
