#!/bin/bash
# Development iteration on one GPU: selected GPU tests (TESTS, default the
# whole -m gpu suite), then bench lines (BENCHES: space-separated config names)
# and a rocprofv3 kernel-stats pass of the first.  Each GPU step has its own
# limit; a fault, abort or timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=gpurun_out/iter
mkdir -p $OUT
source tools/fault_guard.sh
if [ "${TESTS:-all}" != "none" ]; then
  T=${TESTS:-tests}
  [ "$T" = "all" ] && T=tests
  timeout -k 10 600 python -u -m pytest $T -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
  fault_guard $OUT/pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
for cfg in ${BENCHES:-cfg3}; do
  timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-20} --warmup 3 --no-cpu ${BENCH_ARGS:-} > $OUT/bench_$cfg.log 2>&1
  rc=$?; echo "bench $cfg rc=$rc"; tail -1 $OUT/bench_$cfg.log
  fault_guard $OUT/bench_$cfg.log
  [ $rc -ne 0 ] && exit $rc
done
if [ -n "${PROF:-1}" ] && [ "${PROF:-1}" != "0" ]; then
  cfg=$(echo ${BENCHES:-cfg3} | awk '{print $1}')
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/$OUT/prof -o run --output-format csv \
    -- python3 $REPO/bench.py --config $cfg --steps 10 --warmup 2 --no-cpu ${BENCH_ARGS:-} > $REPO/$OUT/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"
  cd $REPO
  fault_guard $OUT/prof.log
  [ $rc -ne 0 ] && exit $rc
  python3 tools/kstats.py $OUT/prof/run_kernel_stats.csv | head -14
fi
exit 0
