# round 6, call h: the N > 1 bench code path end to end on one GPU (host-shm collectives), P = 2, 4, 8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for P in 2 4 8; do
  STEPS=8 bash tools/rehearse_bench_mr.sh $P gpurun_out/r06_rehearsal_mr$P.json || exit 1
done
