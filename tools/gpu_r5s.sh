#!/bin/bash
# Round-5 evidence, part 1: rocprof kernel stats / steady-state means / step
# timelines (cfg3, cfg4, cfg5, cfg2, 8-rank share), the FETCH/WRITE and SQ
# issue passes of the phi kernel (cfg3, cfg4), and the per-rank shares
# (sim-world P = 2, 4, 8 at cfg3, P = 8 at cfg4 and cfg2).
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
source tools/fault_guard.sh
O=gpurun_out/${OUTDIR:-r5s}
mkdir -p $O
STEPS=20 WARMUP=3 TAG=_r5 bash tools/profile.sh > /dev/null || exit 1
fault_guard gpurun_out/prof_r5/bench.log
python3 tools/kstats.py gpurun_out/prof_r5/run_kernel_stats.csv > $O/rocprof_kernel_stats.txt
python3 tools/ktimed.py gpurun_out/prof_r5/run_kernel_trace.csv 3 > $O/rocprof_kernel_timed.txt
python3 tools/step_timeline.py gpurun_out/prof_r5/run_kernel_trace.csv > $O/step_timeline_cfg3.txt
grep "^{" gpurun_out/prof_r5/bench.log | tail -1 > $O/bench_rocprof_run.json
head -4 $O/rocprof_kernel_timed.txt
STEPS=5 WARMUP=2 TAG=_r5cfg4 BENCH_ARGS="--config cfg4 --repeats 1" bash tools/profile.sh > /dev/null || exit 1
python3 tools/ktimed.py gpurun_out/prof_r5cfg4/run_kernel_trace.csv 2 > $O/rocprof_cfg4_kernel_timed.txt
python3 tools/step_timeline.py gpurun_out/prof_r5cfg4/run_kernel_trace.csv > $O/step_timeline_cfg4.txt
head -3 $O/rocprof_cfg4_kernel_timed.txt
STEPS=10 WARMUP=3 TAG=_r5cfg5 BENCH_ARGS="--config cfg5 --repeats 1" bash tools/profile.sh > /dev/null || exit 1
python3 tools/ktimed.py gpurun_out/prof_r5cfg5/run_kernel_trace.csv 3 > $O/rocprof_cfg5_kernel_timed.txt
head -3 $O/rocprof_cfg5_kernel_timed.txt
CONFIGS="cfg2" bash tools/gpu_timeline.sh || exit 1
cp gpurun_out/timeline/cfg2.txt $O/step_timeline_cfg2.txt
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/$O/sim8 -o run --output-format csv \
   -- python3 $REPO/bench.py --sim-world 8 --steps 20 --warmup 3 --no-cpu > $REPO/$O/sim8_prof.log 2>&1) || exit 1
fault_guard $O/sim8_prof.log
python3 tools/step_timeline.py $O/sim8/run_kernel_trace.csv > $O/step_timeline_sim8.txt
tail -1 $O/step_timeline_sim8.txt
TAG=_r5 bash tools/pmc.sh FETCH_SIZE WRITE_SIZE || exit 1
TAG=_r5cfg4 BENCH_ARGS="--config cfg4 --repeats 1" bash tools/pmc.sh FETCH_SIZE WRITE_SIZE || exit 1
TAG=_r5 BENCH_ARGS="--repeats 1 --no-diag" bash tools/pmc_sq.sh "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE" || exit 1
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); dg=d.get('diag_ms_per_step') or {}; h=d['host_ms_per_step']; print('$name', round(d['ms_per_step'],4), 'phi', dg.get('phi_kernel'), 'parts', dg.get('phi_launches_per_step'), 'wait', dg.get('phi_wait_for_g'), 'thr', h.get('threads'), 'trk', d['tracked_brackets'])"
}
for P in 2 4 8; do b sim${P}_cfg3 300 --sim-world $P --steps 20 --warmup 5 --no-cpu; done
SVGD_PHI_SYM=1 b sim8_cfg3_sym 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
b sim8_cfg4 400 --config cfg4 --sim-world 8 --steps 10 --warmup 3 --no-cpu
b sim8_cfg2 300 --config cfg2 --sim-world 8 --steps 20 --warmup 5 --no-cpu
echo r5s done
