#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (one GPU).
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/prof${TAG:-}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv \
    -- python3 "$REPO/bench.py" --steps ${STEPS:-20} --warmup ${WARMUP:-3} --no-cpu ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
find "$OUT" -name "*stats*" | head
exit $rc
