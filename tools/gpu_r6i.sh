# round 6, call i: cfg2 (N = 16384, d = 2) symmetric pass vs row stream, interleaved, with timelines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
source tools/fault_guard.sh
mkdir -p gpurun_out/r6i
for r in 1 2; do
  for v in rows sym; do
    e=0; [ $v = sym ] && e=1
    SVGD_PHI_SYM=$e timeout -k 10 300 python bench.py --config cfg2 --no-cpu --steps 20 --warmup 5 > gpurun_out/r6i/$v.$r.log 2>&1 || exit 1
    fault_guard gpurun_out/r6i/$v.$r.log
    python3 -c "import json; d=json.loads(open('gpurun_out/r6i/$v.$r.log').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],4), [round(x,4) for x in d['repeats']['ms_per_step']], 'phi', round(d['diag_ms_per_step']['phi_kernel'],4), d['roofline']['kernel_launched'])"
  done
done
VARIANTS="rows:SVGD_PHI_SYM=0 sym:SVGD_PHI_SYM=1" CFG=cfg2 bash tools/gpu_tl_var.sh | tail -30
