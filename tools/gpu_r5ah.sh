#!/bin/bash
# Round 5: k_pair_tcol3 (the F32 collect, cfg5) classified by the band's
# centre and half-width (SVGD_TCOL_CLS=2, tcls2.so) vs the lane masks
# (base.so): the collect / F32 parity tests on the variant, interleaved cfg5
# bench A/Bs and rocprof kernel means of both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r5ah
mkdir -p $O
LIB=svgdcpp_amd/libsvgdcpp_amd.so
cp $LIB $O/.cur.so
restore() { cp $O/.cur.so $LIB; }
cp tools/ablibs/tcls2.so $LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_collect.py tests/test_gpu_f32.py tests/test_gpu_f32_accuracy.py tests/test_gpu_track.py tests/test_gpu_fullsize.py \
  > $O/pytest_tcls2.log 2>&1 || { echo "pytest tcls2 failed"; tail -30 $O/pytest_tcls2.log; restore; exit 1; }
fault_guard $O/pytest_tcls2.log
tail -2 $O/pytest_tcls2.log
restore
ROUNDS=3 STEPS=20 BENCH_ARGS="--config cfg5" bash tools/ab_libs.sh base tcls2 > $O/ab_cfg5.txt 2>&1 || { cat $O/ab_cfg5.txt; exit 1; }
cat $O/ab_cfg5.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base tcls2; do
  cp tools/ablibs/$v.so $LIB
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --config cfg5 --steps 10 --warmup 3 --repeats 2 --no-cpu --no-diag > $O/prof_$v.log 2>&1 || { echo "rocprof $v failed"; tail -5 $O/prof_$v.log; restore; exit 1; }
  fault_guard $O/prof_$v.log
done
restore
for v in base tcls2; do
  python3 tools/rocpd_means.py $O/prof_$v/run_results.db "k_pair_tcol3|k_phi_b3|k_compact|k_select_small"
done
echo r5ah done
