#!/bin/bash
# Round-3 final evidence, part 2: the phi kernel's SQ issue counters, the cfg2
# and sim-world-8 step timelines and line, the 8-rank host-shm rehearsal of
# the N > 1 bench path, the per-rank sim-world sweep P = 2, 4, 8
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
source tools/fault_guard.sh
mkdir -p gpurun_out/round
TAG=_r3 bash tools/pmc_sq.sh "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" || exit 1
CONFIGS="cfg2" bash tools/gpu_timeline.sh || exit 1
OUT=$REPO/gpurun_out/timeline
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/sim8 -o run --output-format csv \
   -- python3 $REPO/bench.py --sim-world 8 --steps 20 --warmup 3 --no-cpu > $OUT/sim8.log 2>&1) || exit 1
fault_guard $OUT/sim8.log
python3 tools/step_timeline.py $OUT/sim8/run_kernel_trace.csv > $OUT/sim8.txt
tail -1 $OUT/sim8.txt
timeout -k 10 300 python bench.py --sim-world 8 --steps 20 --warmup 5 --no-cpu > gpurun_out/round/bench_sim8.log 2>&1 || exit 1
tail -1 gpurun_out/round/bench_sim8.log > gpurun_out/round/bench_sim8.json
bash tools/rehearse_bench_mr.sh 8 || exit 1
WORLDS="2 4 8" MULTS="" bash tools/gpu_sim_world.sh || exit 1
echo part2 done
