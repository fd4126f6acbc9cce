#!/bin/bash
# SVGD_TRACK_ERR_MULT 4 (base) / 2.5 / 2 on the other workloads: cfg2, the
# 8-rank cfg3 share, cfg3 with 2, cfg4 (one round each); then the tracking tests under 2.5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4y
mkdir -p $O
b() { local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -3 $O/$name.log; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', round(d['ms_per_step'],4), 'runs', [round(x,4) for x in d['repeats']['ms_per_step']], 'med', round(d['phases_ms_per_step']['median_incl_step_gap'],4), 'trk', d['tracked_brackets'], 'clk', d['gpu_timed'].get('gfxclk_mhz_median'))"; }
for v in X=1 SVGD_TRACK_ERR_MULT=2.5 SVGD_TRACK_ERR_MULT=2; do
  b cfg2_$v $v --config cfg2 --steps 60 --warmup 5 --no-cpu --repeats 3 --no-diag
  b sim8_$v $v --sim-world 8 --steps 40 --warmup 5 --no-cpu --repeats 3 --no-diag
  b cfg3_$v $v --steps 30 --warmup 5 --no-cpu --repeats 3 --no-diag
done
for v in X=1 SVGD_TRACK_ERR_MULT=2.5; do
  b cfg4_$v $v --config cfg4 --steps 8 --warmup 2 --no-cpu --repeats 1 --no-diag
done
SVGD_TRACK_ERR_MULT=2.5 timeout -k 10 400 python -u -m pytest tests/test_gpu_track.py tests/test_gpu_speculative.py tests/test_gpu_fullsize.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest.log
echo r4y done
