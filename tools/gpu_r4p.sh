#!/bin/bash
# k_pair_tcol3 (the F32 bf16-key collect as its own kernel: straight-line
# code per tile kind, entry staging, +inf padding norms) vs the previous
# build (head): the collect + F32 suites on the new build, then interleaved
# cfg5 lines and a rocprof pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4p
mkdir -p $O
LIB=svgdcpp_amd/libsvgdcpp_amd.so
cp $LIB $O/.cur.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_collect.py tests/test_gpu_f32.py tests/test_gpu_median_paths.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest.log; fault_guard $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; cp $O/.cur.so $LIB; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', round(d['ms_per_step'],4), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']], 'med', round(d['phases_ms_per_step']['median_incl_step_gap'],4), 'clk', (d.get('gpu_timed') or {}).get('gfxclk_mhz_median'))"
}
for i in 1 2; do
  for v in head tcol3 tcol3r; do
    cp tools/ablibs/$v.so $LIB
    b ${v}_cfg5_$i 300 --config cfg5 --steps 20 --warmup 3 --no-cpu --repeats 3
  done
done
cp $O/.cur.so $LIB
STEPS=10 WARMUP=3 TAG=_r4p BENCH_ARGS="--config cfg5 --repeats 1" bash tools/profile.sh > /dev/null || exit 1
python3 tools/ktimed.py gpurun_out/prof_r4p/run_kernel_trace.csv 3 > $O/rocprof_cfg5_kernel_timed.txt
head -8 $O/rocprof_cfg5_kernel_timed.txt
echo r4p done
