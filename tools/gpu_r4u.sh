#!/bin/bash
# k_phi_reduce with its weight / optimizer loads ahead of the partial sums:
# row-path parity suites, cfg2 lines; cfg5 with the X mirror forced on (no
# 32 MB X_t copy, the update epilogue writes X_{t+1} to pinned memory).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4u
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host_model_step.py tests/test_gpu_speculative.py tests/test_gpu_fullsize.py tests/test_gpu_matrix_scale.py tests/test_gpu_device_model.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest.log; fault_guard $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
b() { local name=$1; shift; env "$@" timeout -k 10 300 python bench.py $BARGS > $O/$name.log 2>&1 || { echo FAIL $name; tail -3 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); dg=d['diag_ms_per_step']; h=d['host_ms_per_step']; print('$name', round(d['ms_per_step'],4), 'runs', [round(x,4) for x in d['repeats']['ms_per_step']], 'phases', {k: round(v,4) for k,v in d['phases_ms_per_step'].items()}, 'wait_g', round(dg.get('phi_wait_for_g') or 0,4), 'grad', round(h['grad'],3), 'clk', d['gpu_timed'].get('gfxclk_mhz_median'))"; }
for i in 1 2; do
  BARGS="--config cfg2 --steps 40 --warmup 5 --no-cpu --repeats 5" b cfg2.$i X=1
done
for i in 1 2; do
  BARGS="--config cfg5 --steps 20 --warmup 3 --no-cpu --repeats 3" b cfg5_base.$i X=1
  BARGS="--config cfg5 --steps 20 --warmup 3 --no-cpu --repeats 3" b cfg5_mirror.$i SVGD_X_MIRROR=1
done
echo r4u done
