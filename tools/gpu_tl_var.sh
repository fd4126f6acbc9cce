#!/bin/bash
# Step timelines (rocprofv3 kernel trace) of one config under env variants:
# VARIANTS="name:K=V,K2=V2 name2:..." CFG=cfg3 BENCH_ARGS="--sim-world 8"
# -> gpurun_out/tlvar/<name>.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=$REPO/gpurun_out/tlvar
mkdir -p $OUT
source tools/fault_guard.sh
for v in $VARIANTS; do
  name=${v%%:*}; envs=${v#*:}
  (cd /tmp && export TMPDIR=/tmp && for kv in ${envs//,/ }; do [ "$kv" = "-" ] || export "$kv"; done && \
   timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$name -o run --output-format csv \
     -- python3 $REPO/bench.py --config ${CFG:-cfg3} --steps 10 --warmup 3 --no-cpu ${BENCH_ARGS:-} > $OUT/$name.log 2>&1)
  rc=$?; echo "$name rocprof rc=$rc"
  fault_guard $OUT/$name.log
  [ $rc -ne 0 ] && exit $rc
  python3 tools/step_timeline.py $OUT/$name/run_kernel_trace.csv > $OUT/$name.txt
  echo "== $name ($envs)"; cat $OUT/$name.txt
done
echo tlvar done
