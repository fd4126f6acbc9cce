#!/bin/bash
# Round 5: how the median collect depends on the tracked bracket's width --
# per-step prediction errors (SVGD_DEBUG_TRK) at cfg3 and cfg5, and the
# k_pair_mcol / k_pair_tcol3 steady-state means under rocprofv3 at several
# half-width multipliers (SVGD_TRACK_ERR_MULT; a miss redoes the step).
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
source tools/fault_guard.sh
O=gpurun_out/r5d
mkdir -p $O
SVGD_DEBUG_TRK=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --repeats 2 --no-cpu --no-diag > $O/trk_cfg3.log 2>&1 || exit 1
SVGD_DEBUG_TRK=1 timeout -k 10 300 python bench.py --config cfg5 --steps 20 --warmup 3 --repeats 2 --no-cpu --no-diag > $O/trk_cfg5.log 2>&1 || exit 1
fault_guard $O/trk_cfg3.log $O/trk_cfg5.log
grep -c predict $O/trk_cfg3.log; grep "^trk" $O/trk_cfg3.log | tail -8
grep -c predict $O/trk_cfg5.log; grep "^trk" $O/trk_cfg5.log | tail -8
for m in 2.5 1.5 1.0; do
  (cd /tmp && export TMPDIR=/tmp && SVGD_TRACK_ERR_MULT=$m timeout -k 10 300 rocprofv3 --kernel-trace -d $REPO/$O/m$m -o run --output-format csv \
     -- python3 $REPO/bench.py --steps 20 --warmup 3 --repeats 2 --no-cpu --no-diag > $REPO/$O/m$m.log 2>&1) || exit 1
  fault_guard $O/m$m.log
  python3 tools/ktimed.py $O/m$m/run_kernel_trace.csv 3 | grep -E "kernel|mcol|phi_rows<" | head -4
  python3 -c "import json; d=json.load(open('/dev/stdin')); print('mult $m', round(d['ms_per_step'],4), d['tracked_brackets'])" < <(grep '^{' $O/m$m.log | tail -1)
done
echo r5d done
