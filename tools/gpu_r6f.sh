# round 6, call f: k_phi_b3 with two row groups per wave: F32 tests, cfg5 A/B (RG 1 vs 2), cfg3 sanity
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
source tools/fault_guard.sh
mkdir -p gpurun_out/r6f
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_f32.py \
  tests/test_gpu_f32_accuracy.py > gpurun_out/r6f/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r6f/pytest.log; fault_guard gpurun_out/r6f/pytest.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E " gpurun_out/r6f/pytest.log | head; exit $rc; }
b() { local name=$1; shift; timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 "$@" > gpurun_out/r6f/$name.log 2>&1 || exit 1
  fault_guard gpurun_out/r6f/$name.log
  python3 -c "import json; d=json.loads(open('gpurun_out/r6f/$name.log').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step'],4), [round(x,4) for x in d['repeats']['ms_per_step']], 'phi', round(d['diag_ms_per_step']['phi_kernel'],4), 'clk', d['gpu_timed'].get('gfxclk_mhz_median'), d['roofline'].get('kernel_launched'))"; }
for r in 1 2; do
  SVGD_PHI_B3_RG=1 b cfg5_rg1_$r --config cfg5
  SVGD_PHI_B3_RG=2 b cfg5_rg2_$r --config cfg5
done
