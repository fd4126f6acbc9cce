# round 6, call p: the X mirror (update epilogue PCIe writes) vs the copy at
# P = 8 / 4 shares and cfg2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=s8_ ROUNDS=3 BENCH_ARGS="--sim-world 8" bash tools/ab_env.sh on:SVGD_X_MIRROR=1 off:SVGD_X_MIRROR=0 || exit 1
TAG=s4_ ROUNDS=2 BENCH_ARGS="--sim-world 4" bash tools/ab_env.sh on:SVGD_X_MIRROR=1 off:SVGD_X_MIRROR=0 || exit 1
TAG=c2_ ROUNDS=2 STEPS=50 BENCH_ARGS="--config cfg2" bash tools/ab_env.sh on:SVGD_X_MIRROR=1 off:SVGD_X_MIRROR=0 || exit 1
