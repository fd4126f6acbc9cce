#!/bin/bash
# Bitonic select for small buckets: median tests, then the cfg3 kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
source tools/fault_guard.sh
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_median_paths.py tests/test_gpu_speculative.py tests/test_gpu_track.py tests/test_gpu_collect.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_sel2.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab/pytest_sel2.log; fault_guard gpurun_out/ab/pytest_sel2.log; [ $rc -ne 0 ] && exit $rc
CONFIGS="cfg3 cfg2" bash tools/gpu_timeline.sh
for c in cfg3 cfg2; do python3 - gpurun_out/timeline/$c/run_kernel_trace.csv <<'PY'
import csv, sys, statistics
rows=list(csv.DictReader(open(sys.argv[1]))); rows.sort(key=lambda r:int(r['Start_Timestamp']))
v=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows if 'k_select_small' in r['Kernel_Name']]
print(sys.argv[1], 'select us: median', round(statistics.median(v),1), 'max', round(max(v),1), [round(x,1) for x in v[::6]])
PY
done
