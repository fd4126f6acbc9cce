#!/bin/bash
# Round 5: sharded symmetric phi on by default for P <= 4 -- the multi-rank,
# RCCL and symmetric GPU tests, then full-size bench rehearsals (host-shm
# collectives, one GPU) at 2, 4 (symmetric + reduce-scatter) and 8 ranks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r5n
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_gpu_multirank.py tests/test_gpu_rccl.py tests/test_gpu_sym.py tests/test_cpp_api.py > $O/pytest.log 2>&1
rc=$?; fault_guard $O/pytest.log; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "^FAILED|Error" $O/pytest.log | head; exit 1; }
for N in 2 4 8; do
  bash tools/rehearse_bench_mr.sh $N $O/rehearsal_mr$N.json || exit 1
  fault_guard gpurun_out/bench_mr$N.log
done
echo r5n done
