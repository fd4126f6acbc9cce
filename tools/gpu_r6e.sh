# round 6, call e: exp table DMA prologue: sym tests, cfg3 + sim-8 lines, X mirror A/B at sim-8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
source tools/fault_guard.sh
mkdir -p gpurun_out/r6e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sym.py \
  tests/test_gpu_multirank.py -k "symmetric or world8 or sym" > gpurun_out/r6e/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r6e/pytest.log; fault_guard gpurun_out/r6e/pytest.log; [ $rc -eq 0 ] || exit $rc
b() { local name=$1; shift; timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 "$@" > gpurun_out/r6e/$name.log 2>&1 || exit 1
  fault_guard gpurun_out/r6e/$name.log
  python3 -c "import json; d=json.loads(open('gpurun_out/r6e/$name.log').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step'],4), [round(x,4) for x in d['repeats']['ms_per_step']], 'phi', round(d['diag_ms_per_step']['phi_kernel'],4), 'wait', round(d['diag_ms_per_step']['phi_wait_for_g'],4), 'clk', d['gpu_timed'].get('gfxclk_mhz_median'))"; }
for r in 1 2; do
  b cfg3_$r
  b sim8_$r --sim-world 8
  SVGD_X_MIRROR=0 b sim8_nomirror_$r --sim-world 8
done
