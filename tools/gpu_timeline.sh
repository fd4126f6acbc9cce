#!/bin/bash
# Kernel timelines of one steady-state step (rocprofv3 kernel trace) for the
# configs named in CONFIGS; writes gpurun_out/timeline/<cfg>.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=$REPO/gpurun_out/timeline
mkdir -p $OUT
source tools/fault_guard.sh
for cfg in ${CONFIGS:-cfg2 cfg3}; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$cfg -o run --output-format csv \
     -- python3 $REPO/bench.py --config $cfg --steps 10 --warmup 3 --no-cpu ${BENCH_ARGS:-} > $OUT/$cfg.log 2>&1)
  rc=$?; echo "$cfg rocprof rc=$rc"
  fault_guard $OUT/$cfg.log
  [ $rc -ne 0 ] && exit $rc
  python3 tools/step_timeline.py $OUT/$cfg/run_kernel_trace.csv > $OUT/$cfg.txt
  tail -1 $OUT/$cfg.txt
done
exit 0
