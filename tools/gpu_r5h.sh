#!/bin/bash
# Round 5: step timelines with the symmetric phi pass (cfg3, cfg4) and the
# cfg2 one (row stream below N = 32768).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
CONFIGS="cfg3 cfg2" bash tools/gpu_timeline.sh || exit 1
echo r5h done
