#!/bin/bash
# Round evidence on one GPU: the default bench line (with the CPU baseline),
# the rocprofv3 kernel stats of the same command, the two PMC passes of the
# phi kernel's HBM traffic, and the cfg5 (fp32) line.  Outputs are copied to
# profiles/<ROUND>_* by the caller from gpurun_out/round/.
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
source tools/fault_guard.sh
OUT=gpurun_out/round
mkdir -p $OUT
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
fault_guard $OUT/bench.log
tail -1 $OUT/bench.log > $OUT/bench.json
STEPS=20 WARMUP=3 TAG=_round bash tools/profile.sh > /dev/null || exit 1
fault_guard gpurun_out/prof_round/bench.log
cp gpurun_out/prof_round/run_kernel_stats.csv $OUT/rocprof_kernel_stats.csv
python3 tools/kstats.py $OUT/rocprof_kernel_stats.csv > $OUT/rocprof_kernel_stats.txt
# steady state (the 3 warm-up launches of each kernel dropped), as bench.py times it
python3 tools/ktimed.py gpurun_out/prof_round/run_kernel_trace.csv 3 > $OUT/rocprof_kernel_timed.txt
python3 tools/step_timeline.py gpurun_out/prof_round/run_kernel_trace.csv > $OUT/step_timeline.txt
TAG=_round bash tools/pmc.sh FETCH_SIZE WRITE_SIZE || exit 1
timeout -k 10 400 python bench.py --config cfg5 --steps 20 --warmup 3 --no-cpu > $OUT/bench_cfg5.log 2>&1 || exit 1
fault_guard $OUT/bench_cfg5.log
tail -1 $OUT/bench_cfg5.log > $OUT/bench_cfg5.json
STEPS=10 WARMUP=3 TAG=_cfg5 BENCH_ARGS="--config cfg5" bash tools/profile.sh > /dev/null || exit 1
python3 tools/ktimed.py gpurun_out/prof_cfg5/run_kernel_trace.csv 3 > $OUT/rocprof_cfg5_kernel_timed.txt
timeout -k 10 400 python bench.py --config cfg2 --steps 20 --warmup 3 --no-cpu > $OUT/bench_cfg2.log 2>&1 || exit 1
tail -1 $OUT/bench_cfg2.log > $OUT/bench_cfg2.json
echo round profile done
