#!/bin/bash
# Round 5: same-box A/B of the round-4 library (r4) against the current one
# (cur: centring fold, 16-deep reduce loads, AVX-512 gradient, whole-rows
# phi at P = 8), cfg3 and the 8-rank share, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUNDS=2 bash tools/ab_libs.sh r4 cur || exit 1
ROUNDS=2 BENCH_ARGS="--sim-world 8" bash tools/ab_libs.sh r4 cur || exit 1
ROUNDS=1 BENCH_ARGS="--config cfg2" bash tools/ab_libs.sh r4 cur || exit 1
echo r5e done
