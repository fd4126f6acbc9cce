#!/bin/bash
# PMC counters for a short bench (separate passes; counters only with --kernel-trace).
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/pmc${TAG:-}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "${@}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d "$OUT/p$i" -o run --output-format csv \
      -- python3 "$REPO/bench.py" --steps ${STEPS:-2} --warmup 1 --no-cpu ${BENCH_ARGS:-} > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
done
echo pmc done
