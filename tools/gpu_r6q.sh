# round 6, call q: the per-step selected medians of cfg5 and cfg3 (bracket predictor study)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r6q
timeout -k 10 300 python tools/median_trace.py cfg5 130 gpurun_out/r6q/cfg5.json && \
timeout -k 10 300 python tools/median_trace.py cfg3 130 gpurun_out/r6q/cfg3.json
