#!/bin/bash
# Collect pass with the below count on the vector unit (SVGD_MCOL_VCNT=1)
# vs the scalar popcounts (=0): collect / median tests, then rocprof kernel
# means of k_pair_mcol at cfg3 and cfg2 for both builds, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
source tools/fault_guard.sh
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_collect.py tests/test_gpu_median_paths.py tests/test_gpu_track.py tests/test_gpu_speculative.py tests/test_gpu_fullsize.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest.log; fault_guard $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" $O/pytest.log | head; exit $rc; }
LIB=svgdcpp_amd/libsvgdcpp_amd.so
cp $LIB $O/.cur.so
for i in 1 2; do
  for v in vcnt0 vcnt1; do
    for cfg in cfg3 cfg2; do
      cp tools/ablibs/$v.so $LIB
      STEPS=20 WARMUP=3 TAG=_ab_${v}_${cfg}_$i BENCH_ARGS="--config $cfg --repeats 2" bash tools/profile.sh > /dev/null || { cp $O/.cur.so $LIB; exit 1; }
      python3 tools/ktimed.py gpurun_out/prof_ab_${v}_${cfg}_$i/run_kernel_trace.csv 3 > $O/kt_${v}_${cfg}_$i.txt
      echo "$v $cfg $i $(grep k_pair_mcol $O/kt_${v}_${cfg}_$i.txt | cut -c60-) | $(tail -1 gpurun_out/prof_ab_${v}_${cfg}_$i/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4))')"
    done
  done
done
cp $O/.cur.so $LIB
echo r4h done
