#!/bin/bash
# Round 5: the tracked-bracket decisions on cfg5 (SVGD_DEBUG_TRK=1 on stderr).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r5v
mkdir -p $O
SVGD_DEBUG_TRK=1 timeout -k 10 300 python bench.py --config cfg5 --steps 20 --warmup 3 --no-cpu --repeats 2 --no-diag > $O/cfg5.log 2> $O/cfg5.err || { tail -5 $O/cfg5.err; exit 1; }
fault_guard $O/cfg5.err
grep "^trk" $O/cfg5.err | head -60
tail -1 $O/cfg5.log | cut -c1-300
echo r5v done
