# round 6, call o: k_pair_mcol at 5 waves per SIMD (31 KiB LDS, 96 VGPRs, 1280 blocks)
# and the centre form on diagonal tiles: tests, rocprof means, bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
source tools/fault_guard.sh
mkdir -p gpurun_out/r6o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_collect.py tests/test_gpu_track.py tests/test_gpu_median_paths.py tests/test_gpu_parity.py tests/test_gpu_speculative.py tests/test_gpu_multirank.py tests/test_gpu_fullsize.py \
  > gpurun_out/r6o/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6o/pytest.log
fault_guard gpurun_out/r6o/pytest.log
[ $rc -eq 0 ] || exit $rc
cp svgdcpp_amd/libsvgdcpp_amd.so /tmp/r6o_cur.so
for v in wait occ5 d15 wait occ5 d15; do
  cp tools/ablibs/$v.so svgdcpp_amd/libsvgdcpp_amd.so
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r6o/$v" -o run --output-format csv \
      -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/r6o/$v.log" 2>&1 ) || { echo "$v failed"; cp /tmp/r6o_cur.so svgdcpp_amd/libsvgdcpp_amd.so; exit 1; }
  python3 - "$v" <<'PY'
import csv,glob,sys
v=sys.argv[1]
for f in glob.glob(f"gpurun_out/r6o/{v}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mcol" in r["Name"] or "center_d" in r["Name"]:
            print(v, r["Name"][:40], r["Calls"], r["AverageNs"])
PY
done
cp /tmp/r6o_cur.so svgdcpp_amd/libsvgdcpp_amd.so
TAG=c3_ ROUNDS=2 STEPS=30 bash tools/ab_libs.sh wait occ5 d15 || exit 1
TAG=c2_ ROUNDS=2 STEPS=50 BENCH_ARGS="--config cfg2" bash tools/ab_libs.sh wait occ5 d15 || exit 1
TAG=s8_ ROUNDS=2 STEPS=30 BENCH_ARGS="--sim-world 8" bash tools/ab_libs.sh wait occ5 d15 || exit 1
