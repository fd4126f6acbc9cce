#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes of the phi kernels of cfg2, cfg5 and cfg4
# (one pass per counter, short bench runs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=_r4cfg2 BENCH_ARGS="--config cfg2 --repeats 1 --no-diag" bash tools/pmc.sh FETCH_SIZE WRITE_SIZE || exit 1
TAG=_r4cfg5 BENCH_ARGS="--config cfg5 --repeats 1 --no-diag" bash tools/pmc.sh FETCH_SIZE WRITE_SIZE || exit 1
TAG=_r4cfg4 STEPS=1 BENCH_ARGS="--config cfg4 --repeats 1 --no-diag" bash tools/pmc.sh FETCH_SIZE WRITE_SIZE || exit 1
echo r4pmc done
