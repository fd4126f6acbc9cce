#!/bin/bash
# Round 5: k_pair_mcol below count on the vector unit (SVGD_MCOL_CLS=3:
# y = T2 - v sign bytes, v_perm + v_bcnt; cls3.so) vs the centre / half-width
# form with scalar counts (the default, cls2.so) and the lane masks (base.so):
# collect parity tests on cls3, interleaved bench A/Bs at cfg3 and cfg2,
# rocprof kernel means.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r5ai
mkdir -p $O
LIB=svgdcpp_amd/libsvgdcpp_amd.so
cp $LIB $O/.cur.so
restore() { cp $O/.cur.so $LIB; }
cp tools/ablibs/cls3.so $LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_collect.py tests/test_gpu_track.py tests/test_gpu_median_paths.py tests/test_gpu_fullsize.py \
  > $O/pytest_cls3.log 2>&1 || { echo "pytest cls2 failed"; tail -30 $O/pytest_cls3.log; restore; exit 1; }
fault_guard $O/pytest_cls3.log
tail -2 $O/pytest_cls3.log
restore
ROUNDS=3 STEPS=30 bash tools/ab_libs.sh base cls2 cls3 > $O/ab_cfg3.txt 2>&1 || { cat $O/ab_cfg3.txt; exit 1; }
cat $O/ab_cfg3.txt
ROUNDS=3 STEPS=60 BENCH_ARGS="--config cfg2" bash tools/ab_libs.sh base cls2 cls3 > $O/ab_cfg2.txt 2>&1 || { cat $O/ab_cfg2.txt; exit 1; }
cat $O/ab_cfg2.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base cls2 cls3; do
  cp tools/ablibs/$v.so $LIB
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-diag > $O/prof_$v.log 2>&1 || { echo "rocprof $v failed"; tail -5 $O/prof_$v.log; restore; exit 1; }
  fault_guard $O/prof_$v.log
done
restore
for v in base cls2 cls3; do
  python3 tools/rocpd_means.py $O/prof_$v/run_results.db "k_pair_mcol|k_phi_sym|k_compact|k_select_small"
done
echo r5ai done
