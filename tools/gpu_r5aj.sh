#!/bin/bash
# Round 5: k_phi_sym's LDS read order -- the exp-table reads issued before the
# next column's coordinates and the W record (SVGD_SYM_TFIRST=1, tfirst.so) vs
# the shipped order (base.so): the symmetric-pass tests on the variant,
# interleaved cfg3 bench A/Bs and rocprof kernel means.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r5aj
mkdir -p $O
LIB=svgdcpp_amd/libsvgdcpp_amd.so
cp $LIB $O/.cur.so
restore() { cp $O/.cur.so $LIB; }
cp tools/ablibs/tfirst.so $LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sym.py \
  > $O/pytest_tfirst.log 2>&1 || { echo "pytest tfirst failed"; tail -30 $O/pytest_tfirst.log; restore; exit 1; }
fault_guard $O/pytest_tfirst.log
tail -2 $O/pytest_tfirst.log
restore
ROUNDS=4 STEPS=30 bash tools/ab_libs.sh base tfirst > $O/ab_cfg3.txt 2>&1 || { cat $O/ab_cfg3.txt; exit 1; }
cat $O/ab_cfg3.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base tfirst base tfirst; do
  cp tools/ablibs/$v.so $LIB
  rm -rf $O/prof_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-diag > $O/prof_$v.log 2>&1 || { echo "rocprof $v failed"; tail -5 $O/prof_$v.log; restore; exit 1; }
  fault_guard $O/prof_$v.log
  python3 tools/rocpd_means.py $O/prof_$v/run_results.db "k_phi_sym|k_pair_mcol"
done
restore
echo r5aj done
