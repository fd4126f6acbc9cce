# round 6, call k: the collect's split-bf16 operands written by the centring
# (tests, then same-box A/B base vs split at cfg3 and cfg2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
source tools/fault_guard.sh
mkdir -p gpurun_out/r6k
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_collect.py tests/test_gpu_track.py tests/test_gpu_median_paths.py tests/test_gpu_parity.py \
  > gpurun_out/r6k/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6k/pytest.log
fault_guard gpurun_out/r6k/pytest.log
[ $rc -eq 0 ] || exit $rc
cp svgdcpp_amd/libsvgdcpp_amd.so /tmp/r6k_cur.so && cp tools/ablibs/code1.so svgdcpp_amd/libsvgdcpp_amd.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_collect.py tests/test_gpu_track.py > gpurun_out/r6k/pytest_code1.log 2>&1
rc=$?; cp /tmp/r6k_cur.so svgdcpp_amd/libsvgdcpp_amd.so; echo "code1 pytest rc=$rc"; tail -2 gpurun_out/r6k/pytest_code1.log
fault_guard gpurun_out/r6k/pytest_code1.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=3 STEPS=30 bash tools/ab_libs.sh base split code1 || exit 1
ROUNDS=2 STEPS=50 BENCH_ARGS="--config cfg2" bash tools/ab_libs.sh base split code1 || exit 1
