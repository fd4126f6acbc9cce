#!/bin/bash
# Multi-rank bench rehearsal on ONE GPU: torch.distributed.run with N ranks on
# device 0, collectives through the host shared-memory backend (RCCL refuses
# two ranks on one device).  Checks the N>1 bench code path end to end (gloo
# barrier, max-over-ranks timing, one JSON line from rank 0, every rank's
# per_rank record) on the default per-rank path -- at N >= 4 phi + update in
# two row parts, the X mirror, speculative steps with tracked brackets -- and
# every step's collective sequence compared across ranks (SVGD_DEBUG_COLL=1).
# The timing itself is meaningless (N ranks share one GPU).
#   tools/rehearse_bench_mr.sh N [out.json]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=${1:-2}
OUT=${2:-gpurun_out/bench_mr$N.json}
SVGD_BENCH_DEVICE=0 SVGD_HOSTCOMM=svgd_bench_$$ SVGD_DEBUG_COLL=1 OMP_NUM_THREADS=4 timeout -k 10 400 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus $N --steps ${STEPS:-8} --warmup 2 --repeats 2 ${BENCH_ARGS:-} > gpurun_out/bench_mr$N.log 2>&1 || { tail -20 gpurun_out/bench_mr$N.log; exit 1; }
grep '^{"metric"' gpurun_out/bench_mr$N.log | tail -1 > $OUT
python3 - "$OUT" "$N" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); n = int(sys.argv[2])
pr = d["per_rank"]
rows = [(r["rank"], r["rows"], r["diag_ms_per_step"]["phi_launches_per_step"], r["n_ranks_seen"],
         r["tracked_brackets"], r.get("phi_kernel")) for r in pr]
print("n_gpus", d["n_gpus"], "ranks", len(pr), "env", d.get("env_knobs"))
for r in rows:
    print("rank %d rows %d phi_launches %d ranks_seen %d trk %s phi %s" % r)
assert d["n_gpus"] == n and len(pr) == n and all(r[3] == n for r in rows)
PY
