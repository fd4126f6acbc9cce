cd "${GRAFT_REPO_ROOT}"
REPO=$(pwd); OUT=$REPO/gpurun_out/exp; mkdir -p $OUT
for spec in 1 0; do
  (cd /tmp && export TMPDIR=/tmp && SVGD_SPECULATE=$spec timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/s$spec -o run --output-format csv -- python3 $REPO/bench.py --config cfg3 --steps 6 --warmup 2 --no-cpu > $OUT/s$spec.log 2>&1) || exit 1
  python3 tools/step_timeline.py $OUT/s$spec/run_kernel_trace.csv > $OUT/s$spec.txt
  echo "spec=$spec"; head -5 $OUT/s$spec.txt; tail -1 $OUT/s$spec.txt
done
ls $OUT/s1
