#!/bin/bash
# phi column splits: 3 blocks per resident slot against 2 (cfg3, and the 8-rank share)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
VARIANTS="base SVGD_PHI_SPLIT_MULT=3" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
VARIANTS="base SVGD_PHI_SPLIT_MULT=3" BENCH_ARGS="--sim-world 8" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
