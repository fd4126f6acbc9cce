#!/bin/bash
# Interleaved MFMA chains in k_pair_mcol: collect tests, kernel traces, lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
source tools/fault_guard.sh
timeout -k 10 900 python -u -m pytest tests/test_gpu_collect.py tests/test_gpu_fullsize.py tests/test_gpu_median_paths.py tests/test_gpu_track.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_il.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab/pytest_il.log; fault_guard gpurun_out/ab/pytest_il.log; [ $rc -ne 0 ] && exit $rc
CONFIGS="cfg3 cfg2" bash tools/gpu_timeline.sh
for c in cfg3 cfg2; do python3 - gpurun_out/timeline/$c/run_kernel_trace.csv <<'PY'
import csv, sys, statistics
rows=list(csv.DictReader(open(sys.argv[1])))
v=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows if 'k_pair_mcol' in r['Kernel_Name']]
print(sys.argv[1], 'mcol us: median', round(statistics.median(v[3:]),1), 'min', round(min(v),1))
PY
done
VARIANTS="base" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
