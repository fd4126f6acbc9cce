#!/bin/bash
# Round 5, first GPU pass: the changed / new GPU tests (row-part multi-rank
# path, split G communicator, fp32 accuracy, mirror, resume), then the whole
# GPU suite, the 8-rank bench rehearsal on the default path, a cfg3 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r5a
mkdir -p $O
T="python -u -m pytest -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $T -v -s tests/test_gpu_multirank.py tests/test_gpu_rccl.py tests/test_gpu_f32_accuracy.py \
  tests/test_gpu_host_model_step.py tests/test_cpp_api.py > $O/pytest_new.log 2>&1; rc=$?
echo "new tests rc=$rc"; tail -3 $O/pytest_new.log; fault_guard $O/pytest_new.log
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest_new.log | head -20; exit $rc; }
grep -E "b3 |keys b3|cfg5 rows" $O/pytest_new.log | head -12
timeout -k 10 900 $T -q tests > $O/pytest_gpu.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -2 $O/pytest_gpu.log; fault_guard $O/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $O/pytest_gpu.log | head; exit $rc; }
bash tools/rehearse_bench_mr.sh 8 $O/rehearsal_mr8.json || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
fault_guard $O/bench.log
tail -1 $O/bench.log > $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); print('cfg3', round(d['ms_per_step'],4), d['value'], d['roofline']['frac'], d['cpu_baseline']['accuracy'], d['env_knobs'])"
(cd build && timeout -k 10 300 ./svgd_run_bench > ../$O/bench_cpp.log 2>&1) || { tail -5 $O/bench_cpp.log; exit 1; }
fault_guard $O/bench_cpp.log
grep '^{' $O/bench_cpp.log | tail -1 > $O/bench_cpp.json; cut -c1-400 $O/bench_cpp.json
echo r5a done
