#!/bin/bash
# Round 5: the symmetric phi pass as the default (one rank, d <= 8): the GPU
# suite, then same-box A/B against the row stream (SVGD_PHI_SYM=0) at cfg2,
# cfg3 and cfg4 (one GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r5g
mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -q tests \
  > $O/pytest_gpu.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -2 $O/pytest_gpu.log; fault_guard $O/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; }
VARIANTS="base SVGD_PHI_SYM=0" BENCH_ARGS="--config cfg2" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
VARIANTS="base SVGD_PHI_SYM=0" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
for v in base SVGD_PHI_SYM=0; do
  if [ "$v" = base ]; then envs=""; else envs="$v"; fi
  env $envs timeout -k 10 600 python bench.py --config cfg4 --steps 5 --warmup 2 --repeats 2 --no-cpu > $O/cfg4_$v.log 2>&1 || { tail -5 $O/cfg4_$v.log; exit 1; }
  fault_guard $O/cfg4_$v.log
  tail -1 $O/cfg4_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg4 $v', round(d['ms_per_step'],3), d['roofline']['kernel_launched'], round(d['roofline']['avg_launch_ms'],3))"
done
echo r5g done
