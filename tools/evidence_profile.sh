#!/bin/bash
# Round evidence, part 1 (R=<round tag>, e.g. R=r06): rocprof kernel stats,
# steady-state means and step timelines (cfg3, cfg4, cfg5, cfg2, the 8-rank
# share), the FETCH/WRITE and SQ issue passes of the phi kernel (cfg3,
# cfg4), and the per-rank shares (sim-world P = 2, 4, 8 at cfg3, P = 8 at
# cfg4 and cfg2).  PARTS selects a subset: prof cfg4 cfg5 cfg2 sim8tl pmc sim.
#   R=r06 bash tools/evidence_profile.sh  -> gpurun_out/<R>s/
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
source tools/fault_guard.sh
R=${R:-rXX}
O=gpurun_out/${R}s
PARTS=${PARTS:-"prof cfg4 cfg5 cfg2 sim8tl pmc sim"}
mkdir -p $O
has() { [[ " $PARTS " == *" $1 "* ]]; }
if has prof; then
  STEPS=20 WARMUP=3 TAG=_$R bash tools/profile.sh > /dev/null || exit 1
  fault_guard gpurun_out/prof_$R/bench.log
  python3 tools/kstats.py gpurun_out/prof_$R/run_kernel_stats.csv > $O/rocprof_kernel_stats.txt
  cp gpurun_out/prof_$R/run_kernel_stats.csv $O/rocprof_kernel_stats.csv
  python3 tools/ktimed.py gpurun_out/prof_$R/run_kernel_trace.csv 3 > $O/rocprof_kernel_timed.txt
  python3 tools/step_timeline.py gpurun_out/prof_$R/run_kernel_trace.csv > $O/step_timeline_cfg3.txt
  grep "^{" gpurun_out/prof_$R/bench.log | tail -1 > $O/bench_rocprof_run.json
  head -4 $O/rocprof_kernel_timed.txt
fi
if has cfg4; then
  STEPS=5 WARMUP=2 TAG=_${R}cfg4 BENCH_ARGS="--config cfg4 --repeats 1" bash tools/profile.sh > /dev/null || exit 1
  python3 tools/ktimed.py gpurun_out/prof_${R}cfg4/run_kernel_trace.csv 2 > $O/rocprof_cfg4_kernel_timed.txt
  python3 tools/step_timeline.py gpurun_out/prof_${R}cfg4/run_kernel_trace.csv > $O/step_timeline_cfg4.txt
  head -3 $O/rocprof_cfg4_kernel_timed.txt
fi
if has cfg5; then
  STEPS=10 WARMUP=3 TAG=_${R}cfg5 BENCH_ARGS="--config cfg5 --repeats 1" bash tools/profile.sh > /dev/null || exit 1
  python3 tools/ktimed.py gpurun_out/prof_${R}cfg5/run_kernel_trace.csv 3 > $O/rocprof_cfg5_kernel_timed.txt
  head -3 $O/rocprof_cfg5_kernel_timed.txt
fi
if has cfg2; then
  CONFIGS="cfg2" bash tools/gpu_timeline.sh || exit 1
  cp gpurun_out/timeline/cfg2.txt $O/step_timeline_cfg2.txt
fi
if has sim8tl; then
  for form in default rows; do
    envs=""; [ $form = rows ] && envs="SVGD_PHI_SYM=0"
    (cd /tmp && export TMPDIR=/tmp && for kv in $envs; do export "$kv"; done && \
     timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/$O/sim8_$form -o run --output-format csv \
       -- python3 $REPO/bench.py --sim-world 8 --steps 20 --warmup 3 --no-cpu > $REPO/$O/sim8_${form}_prof.log 2>&1) || exit 1
    fault_guard $O/sim8_${form}_prof.log
    python3 tools/step_timeline.py $O/sim8_$form/run_kernel_trace.csv > $O/step_timeline_sim8_$form.txt
    tail -1 $O/step_timeline_sim8_$form.txt
  done
fi
if has pmc; then
  TAG=_$R bash tools/pmc.sh FETCH_SIZE WRITE_SIZE || exit 1
  TAG=_${R}cfg4 BENCH_ARGS="--config cfg4 --repeats 1" bash tools/pmc.sh FETCH_SIZE WRITE_SIZE || exit 1
  TAG=_$R BENCH_ARGS="--repeats 1 --no-diag" bash tools/pmc_sq.sh "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE" || exit 1
fi
if has sim; then
  b() { # name timeout args...
    local name=$1 t=$2; shift 2
    timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
    fault_guard $O/$name.log
    tail -1 $O/$name.log > $O/$name.json
    python3 -c "import json,sys; d=json.load(open('$O/$name.json')); dg=d.get('diag_ms_per_step') or {}; h=d['host_ms_per_step']; print('$name', round(d['ms_per_step'],4), 'phi', dg.get('phi_kernel'), 'parts', dg.get('phi_launches_per_step'), 'wait', dg.get('phi_wait_for_g'), 'thr', h.get('threads'), 'trk', d['tracked_brackets'], d.get('phi_kernel'))"
  }
  for P in 2 4 8; do b sim${P}_cfg3 300 --sim-world $P --steps 20 --warmup 5 --no-cpu; done
  SVGD_PHI_SYM=1 b sim8_cfg3_sym 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
  SVGD_PHI_SYM=0 b sim8_cfg3_rows 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
  SVGD_HOST_THREADS=2 b sim8_cfg3_2thr 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
  b sim8_cfg4 400 --config cfg4 --sim-world 8 --steps 10 --warmup 3 --no-cpu
  b sim8_cfg2 300 --config cfg2 --sim-world 8 --steps 20 --warmup 5 --no-cpu
fi
echo "evidence_profile $R done"
