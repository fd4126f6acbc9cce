#!/bin/bash
# XCD-aligned column splits (S = 8: block b runs on XCD b % 8 = its split, so
# an XCD reads 1/8 of the columns): A/B against S = 2 and the HBM traffic of
# both (FETCH_SIZE, WRITE_SIZE passes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
VARIANTS="base SVGD_PHI_SPLIT_MULT=8" SKIP_PYTEST=1 bash tools/gpu_ab_phi.sh || exit 1
TAG=_s2 bash tools/pmc.sh FETCH_SIZE WRITE_SIZE || exit 1
SVGD_PHI_SPLIT_MULT=8 TAG=_s8 bash tools/pmc.sh FETCH_SIZE WRITE_SIZE || exit 1
