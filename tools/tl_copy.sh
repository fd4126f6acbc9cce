cd "${GRAFT_REPO_ROOT}"
REPO=$(pwd); OUT=$REPO/gpurun_out/tlc; mkdir -p $OUT
for cfg in cfg2 cfg3; do
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/$cfg -o run --output-format csv -- python3 $REPO/bench.py --config $cfg --steps 10 --warmup 3 --no-cpu > $OUT/$cfg.log 2>&1) || exit 1
python3 tools/step_timeline.py $OUT/$cfg/run_kernel_trace.csv $OUT/$cfg/run_memory_copy_trace.csv > $OUT/$cfg.txt || exit 1
done
