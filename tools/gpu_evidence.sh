#!/bin/bash
# Counter evidence for the fp64 design: the MFMA/VALU co-issue
# micro-benchmark, the available counter list, and SQ passes over a short cfg3
# bench (k_phi_rows, k_pair_rows).  One counter pass per rocprofv3 run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=$REPO/gpurun_out/evidence${TAG:-}
mkdir -p $OUT
source tools/fault_guard.sh
if [ -z "$NOUBENCH" ]; then
  timeout -k 10 120 ./tools/ubench_f64 > $OUT/ubench_f64.txt 2>&1 || { cat $OUT/ubench_f64.txt; exit 1; }
  cat $OUT/ubench_f64.txt
fi
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set -d "$OUT/p$i" -o run --output-format csv \
      -- python3 "$REPO/bench.py" --steps 2 --warmup 1 --no-cpu ${BENCH_ARGS:-} > "$OUT/p$i.log" 2>&1
  rc=$?
  fault_guard "$OUT/p$i.log"
  if [ $rc -ne 0 ]; then echo "pass $i ($set) rc=$rc"; tail -3 "$OUT/p$i.log"; [ $rc -ge 124 ] && exit $rc; fi
done
echo evidence done
