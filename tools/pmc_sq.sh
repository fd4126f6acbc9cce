#!/bin/bash
# SQ issue/stall counters for the hot kernels of a short bench (one pass per
# counter set; at most 8 SQ counters per pass).  Also lists the counters.
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc_sq${TAG:-}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d "$OUT/p$i" -o run --output-format csv \
      -- python3 "$REPO/bench.py" --steps 2 --warmup 1 --no-cpu ${BENCH_ARGS:-} > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
echo pmc_sq done
