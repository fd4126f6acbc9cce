#!/bin/bash
# Round 5: step timelines of the P = 8 share (sim-world 8, cfg3), row stream
# vs the sharded symmetric pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=$REPO/gpurun_out/r5l
mkdir -p $OUT
source tools/fault_guard.sh
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_sym.py "tests/test_gpu_multirank.py::test_sharded_symmetric_phi" > $OUT/pytest.log 2>&1
rc=$?; fault_guard $OUT/pytest.log; tail -3 $OUT/pytest.log; [ $rc = 0 ] || exit 1
for v in ${VARIANTS:-rows:0 sym:1}; do
  name=${v%%:*}; val=${v##*:}
  (cd /tmp && export TMPDIR=/tmp SVGD_PHI_SYM=$val && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$name -o run --output-format csv \
     -- python3 $REPO/bench.py --config cfg3 --sim-world 8 --steps 10 --warmup 3 --no-cpu > $OUT/$name.log 2>&1)
  rc=$?; echo "$name rocprof rc=$rc"
  fault_guard $OUT/$name.log
  [ $rc -ne 0 ] && exit $rc
  python3 tools/step_timeline.py $OUT/$name/run_kernel_trace.csv > $OUT/$name.txt
  cat $OUT/$name.txt
done
echo r5l done
