#!/bin/bash
# Multi-rank bench rehearsal on ONE GPU: torch.distributed.run with N ranks on
# device 0, collectives through the host shared-memory backend (RCCL refuses
# two ranks on one device).  Checks the N>1 bench code path end to end (gloo
# barrier, max-over-ranks timing, one JSON line from rank 0); the timing itself
# is meaningless (N ranks share one GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=${1:-2}
SVGD_BENCH_DEVICE=0 SVGD_HOSTCOMM=svgd_bench_$$ OMP_NUM_THREADS=4 timeout -k 10 300 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus $N --steps 3 --warmup 1 > gpurun_out/bench_mr$N.log 2>&1 || { tail -20 gpurun_out/bench_mr$N.log; exit 1; }
grep '"metric"' gpurun_out/bench_mr$N.log | tail -1 | cut -c1-200
