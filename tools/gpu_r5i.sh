#!/bin/bash
# Round 5: symmetric pass without the row-record prep launch and with the
# batched finish -- its parity tests, the step timeline, A/B vs sym1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
mkdir -p gpurun_out/r5i
timeout -k 10 600 python -u -m pytest tests/test_gpu_sym.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_speculative.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r5i/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 gpurun_out/r5i/pytest.log; fault_guard gpurun_out/r5i/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" gpurun_out/r5i/pytest.log | head; exit $rc; }
CONFIGS="cfg3" bash tools/gpu_timeline.sh || exit 1
cat gpurun_out/timeline/cfg3.txt
ROUNDS=2 bash tools/ab_libs.sh new sym2 || exit 1
echo r5i done
