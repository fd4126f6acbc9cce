#!/bin/bash
# Round 5: (1) the symmetric phi pass with 16-byte record reads (SVGD_PHI_SYM=1)
# against the row stream, same box, with its parity tests (tests/test_gpu_sym.py
# first); (2) the unrolled collect (new) against the previous build (cur).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_sym.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/ab/pytest_sym.log 2>&1; rc=$?
echo "sym tests rc=$rc"; tail -1 gpurun_out/ab/pytest_sym.log; fault_guard gpurun_out/ab/pytest_sym.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="base SVGD_PHI_SYM=1" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
ROUNDS=2 bash tools/ab_libs.sh cur new || exit 1
echo r5f done
