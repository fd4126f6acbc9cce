#!/bin/bash
# Final round-3 checks: the driver's own commands (smoke, default bench line),
# then the evidence script, then the per-rank sim-world sweep P = 2, 4, 8
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
source tools/fault_guard.sh
mkdir -p gpurun_out/round
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round/smoke.log 2>&1 || { tail -5 gpurun_out/round/smoke.log; exit 1; }
tail -1 gpurun_out/round/smoke.log
start=$(date +%s)
timeout -k 10 600 python bench.py > gpurun_out/round/bench_default.log 2>&1 || { tail -5 gpurun_out/round/bench_default.log; exit 1; }
echo "default bench took $(( $(date +%s) - start )) s"
tail -1 gpurun_out/round/bench_default.log > gpurun_out/round/bench_default.json
bash tools/gpu_evidence_r3.sh || exit 1
WORLDS="2 4 8" MULTS="" bash tools/gpu_sim_world.sh
