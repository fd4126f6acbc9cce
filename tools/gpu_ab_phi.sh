#!/bin/bash
# A/B of phi-kernel variants (env knobs) on one box: interleaved cfg3 bench
# lines (no CPU leg), then the d = 8 parity tests under each variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
source tools/fault_guard.sh
VARIANTS=${VARIANTS:-"base SVGD_PHI_SMEM=4 SVGD_PHI_SMEM=5"}
for round in 1 2; do
  for v in $VARIANTS; do
    if [ "$v" = base ]; then envs=""; else envs="$v"; fi
    env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab/$v.$round${BENCH_ARGS// /_}.log 2>&1 || { echo "FAIL $v"; tail -3 gpurun_out/ab/$v.$round${BENCH_ARGS// /_}.log; exit 1; }
    fault_guard gpurun_out/ab/$v.$round${BENCH_ARGS// /_}.log
    python3 - "$v" gpurun_out/ab/$v.$round${BENCH_ARGS// /_}.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().split("\n")[-1])
print(f"{sys.argv[1]:24s} ms/step {d['ms_per_step']:.3f} runs {[round(x,3) for x in d['repeats']['ms_per_step']]} phi_kernel {d['roofline']['avg_launch_ms']:.4f} clk {d['gpu_diag'].get('gfxclk_mhz_median')} pw {d['gpu_diag'].get('power_w_median')}")
PY
  done
done
[ -n "$SKIP_PYTEST" ] && exit 0
for v in $VARIANTS; do
  [ "$v" = base ] && continue
  env $v timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_speculative.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_$v.log 2>&1
  rc=$?; echo "pytest $v rc=$rc"; tail -1 gpurun_out/ab/pytest_$v.log
  fault_guard gpurun_out/ab/pytest_$v.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
