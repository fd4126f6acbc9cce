#!/bin/bash
# Per-rank step of a P-GPU run, simulated on one GPU (SVGD_SIM_WORLD: rank 0's
# rows and pair share, no collectives): P = 1, 2, 4, 8 at cfg3, plus knob A/Bs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sim
source tools/fault_guard.sh
run() { # name env... -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu "$@" > gpurun_out/sim/$name.log 2>&1 || { echo "FAIL $name"; tail -3 gpurun_out/sim/$name.log; exit 1; }
  fault_guard gpurun_out/sim/$name.log
  python3 - "$name" gpurun_out/sim/$name.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().split("\n")[-1])
dg = d.get("diag_ms_per_step") or {}
print(f"{sys.argv[1]:22s} ms/step {d['ms_per_step']:.3f} phi_kernel {dg.get('phi_kernel', 0):.4f} phases {json.dumps({k: round(v, 4) for k, v in d['phases_ms_per_step'].items()})} path {d['median_path']} clk {d['gpu_diag'].get('gfxclk_mhz_median')}")
PY
}
for P in ${WORLDS:-1 2 4 8}; do run sim$P X=1 -- --sim-world $P || exit 1; done
for m in ${MULTS:-1 4}; do run sim8_mult$m SVGD_PHI_SPLIT_MULT=$m -- --sim-world 8 || exit 1; done
exit 0
