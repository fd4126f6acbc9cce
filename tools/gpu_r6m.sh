# round 6, call m: exact three-part bf16 split in the collect (margin 2^-17
# nmax): tests, rocprof kernel means split2 vs split3, bench A/B cfg3 / cfg2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
source tools/fault_guard.sh
mkdir -p gpurun_out/r6m
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_collect.py tests/test_gpu_track.py tests/test_gpu_median_paths.py tests/test_gpu_parity.py tests/test_gpu_speculative.py \
  > gpurun_out/r6m/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6m/pytest.log
fault_guard gpurun_out/r6m/pytest.log
[ $rc -eq 0 ] || exit $rc
cp svgdcpp_amd/libsvgdcpp_amd.so /tmp/r6m_cur.so
for v in split2 split3 split2 split3; do
  cp tools/ablibs/$v.so svgdcpp_amd/libsvgdcpp_amd.so
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r6m/$v" -o run --output-format csv \
      -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/r6m/$v.log" 2>&1 ) || { echo "$v failed"; cp /tmp/r6m_cur.so svgdcpp_amd/libsvgdcpp_amd.so; exit 1; }
  python3 - "$v" <<'PY'
import csv,glob,sys
v=sys.argv[1]
for f in glob.glob(f"gpurun_out/r6m/{v}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mcol" in r["Name"] or "center_d" in r["Name"]:
            print(v, r["Name"][:40], r["Calls"], r["AverageNs"])
PY
done
cp /tmp/r6m_cur.so svgdcpp_amd/libsvgdcpp_amd.so
TAG=c3_ ROUNDS=2 STEPS=30 bash tools/ab_libs.sh split2 split3 || exit 1
TAG=c2_ ROUNDS=2 STEPS=50 BENCH_ARGS="--config cfg2" bash tools/ab_libs.sh split2 split3 || exit 1
