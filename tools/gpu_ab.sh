#!/bin/bash
# One GPU call of a same-box A/B: the GPU tests TESTS against the current
# library, then for each library variant in VARIANTS (tools/ablibs/<v>.so,
# built by tools/build_collect_variant.sh or from a git revision) the rocprof
# means of the kernels matching KERNELS and bench lines at each of CONFIGS
# (cfg3 | cfg2 | cfg5 | sim8 ...), ROUNDS interleaved passes.
#   TESTS="tests/test_gpu_collect.py" VARIANTS="base exp" CONFIGS="cfg3 cfg2" \
#     TAG=r6x /usr/local/graft/bin/gpurun -- bash tools/gpu_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log
  fault_guard $OUT/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
[ -n "${VARIANTS:-}" ] || exit 0
cp svgdcpp_amd/libsvgdcpp_amd.so /tmp/gpu_ab_cur.so
restore() { cp /tmp/gpu_ab_cur.so svgdcpp_amd/libsvgdcpp_amd.so; }
if [ -n "${KERNELS:-}" ]; then
  for v in $VARIANTS; do
    cp tools/ablibs/$v.so svgdcpp_amd/libsvgdcpp_amd.so
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_$v" -o run \
        --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/$OUT/prof_$v.log" 2>&1 ) \
      || { echo "$v rocprof failed"; restore; exit 1; }
    fault_guard $OUT/prof_$v.log
    python3 - "$OUT/prof_$v" "$v" "$KERNELS" <<'PY'
import csv, glob, re, sys
d, v, pat = sys.argv[1:4]
for f in glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if re.search(pat, r["Name"]):
            print(v, r["Name"][:48], r["Calls"], r["AverageNs"])
PY
  done
fi
for cfg in ${CONFIGS:-cfg3}; do
  case $cfg in
    sim*) args="--sim-world ${cfg#sim}" ;;
    *) args="--config $cfg" ;;
  esac
  TAG=${cfg}_ ROUNDS=${ROUNDS:-2} STEPS=${STEPS:-30} BENCH_ARGS="$args" bash tools/ab_libs.sh $VARIANTS || { restore; exit 1; }
done
restore
