#!/bin/bash
# A/B timing of library builds on one box: each tools/ablibs/<name>.so is put
# in place of svgdcpp_amd/libsvgdcpp_amd.so in turn (ROUNDS passes, so box
# drift shows), one bench line each.  The current library is restored after.
# Usage: bash tools/ab_libs.sh base exp4096 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
source tools/fault_guard.sh
LIB=svgdcpp_amd/libsvgdcpp_amd.so
cp $LIB /tmp/ab_cur.so
for round in $(seq ${ROUNDS:-2}); do
  for v in "$@"; do
    cp tools/ablibs/$v.so $LIB
    timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab/${TAG:-}$v.$round.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab/${TAG:-}$v.$round.log; cp /tmp/ab_cur.so $LIB; exit 1; }
    fault_guard gpurun_out/ab/${TAG:-}$v.$round.log
    tail -1 gpurun_out/ab/${TAG:-}$v.$round.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step'],3), {k: round(x,3) for k,x in d['phases_ms_per_step'].items() if isinstance(x, float)})"
  done
done
cp /tmp/ab_cur.so $LIB
