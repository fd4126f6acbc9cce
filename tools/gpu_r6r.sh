# round 6, call r: bracket predictor = the narrower of the quadratic / cubic
# extrapolation: tracking tests, then A/B base vs trk at cfg3, cfg5, cfg2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TESTS="tests/test_gpu_track.py tests/test_gpu_speculative.py tests/test_gpu_median_paths.py tests/test_gpu_rccl.py tests/test_gpu_multirank.py" \
  VARIANTS="base trk" CONFIGS="cfg3 cfg5 cfg2" ROUNDS=2 STEPS=60 TAG=r6r bash tools/gpu_ab.sh
