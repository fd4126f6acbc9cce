#!/bin/bash
# Bracket sample size A/B at cfg3 (SVGD_MEDIAN_SAMPLE): ms/step and the median
# phase per size, sizes interleaved over two rounds (box drift shows as a
# round-to-round difference).  Each run has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sample_ab
source tools/fault_guard.sh
for rep in 1 2; do
  for s in ${SIZES:-1048576 2097152 4194304}; do
    log=gpurun_out/sample_ab/${CFG:-cfg3}_${s}_$rep.log
    SVGD_MEDIAN_SAMPLE=$s timeout -k 10 200 python bench.py --config ${CFG:-cfg3} --steps 20 --warmup 3 --no-cpu > $log 2>&1 || exit $?
    fault_guard $log
    tail -1 $log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('S=$s rep $rep', round(d['ms_per_step'], 4), {k: round(v, 4) for k, v in d['phases_ms_per_step'].items()})"
  done
done
