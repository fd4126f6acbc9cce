#!/bin/bash
# Round 4, first GPU call: the suite, a bench line for every BASELINE config
# (cpu_baseline on each), the per-rank share of P = 2/4/8 (cfg3) and P = 8
# (cfg4) with the host-gradient threads a real rank gets (cgroup quota / P),
# and rocprof kernel means of cfg4 on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4a
mkdir -p $O
nproc > $O/nproc.txt; cat /sys/fs/cgroup/cpu.max >> $O/nproc.txt 2>/dev/null
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest_gpu.log; fault_guard $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" $O/pytest_gpu.log | head; exit $rc; }
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log > $O/$name.json
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); r=d['roofline']; print('$name', round(d['ms_per_step'],4), 'frac', r.get('frac'), 'cpu', (d.get('cpu_baseline') or {}).get('value'), 'wait', (d.get('diag_ms_per_step') or {}).get('phi_wait_for_g'), 'thr', d['host_ms_per_step'].get('threads'))"
}
b cfg3 600 --steps 20 --warmup 3
b cfg2 400 --config cfg2 --steps 20 --warmup 3
b cfg5 500 --config cfg5 --steps 20 --warmup 3
b cfg4 900 --config cfg4 --steps 5 --warmup 2 --repeats 3
for P in 2 4 8; do b sim${P}_cfg3 300 --sim-world $P --steps 20 --warmup 5 --no-cpu; done
b sim8_cfg4 400 --config cfg4 --sim-world 8 --steps 10 --warmup 3 --no-cpu
SVGD_HOST_THREADS=8 b sim8_cfg3_t8 300 --sim-world 8 --steps 20 --warmup 5 --no-cpu
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_cfg4 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg4 --steps 5 --warmup 2 --repeats 1 --no-cpu > $GRAFT_REPO_ROOT/$O/prof_cfg4.log 2>&1 || { echo "rocprof cfg4 failed"; tail -5 $GRAFT_REPO_ROOT/$O/prof_cfg4.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 tools/ktimed.py $O/prof_cfg4/run_kernel_trace.csv 2 > $O/rocprof_cfg4_kernel_timed.txt
head -8 $O/rocprof_cfg4_kernel_timed.txt
echo r4a done
