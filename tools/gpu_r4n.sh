#!/bin/bash
# Same-box A/B of collect variants (tools/ablibs, built from the working
# tree): tcol0 = the default build; tcolpipe = k_pair_tcol<64> with the row
# parts of row block rb + 1 read before rb's MFMAs (cfg5); clsv = k_pair_mcol
# classifying by sign bits on the vector unit (SVGD_MCOL_CLS=1; cfg3, cfg2),
# then the collect suite under clsv.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4n
mkdir -p $O
LIB=svgdcpp_amd/libsvgdcpp_amd.so
cp $LIB $O/.cur.so
b() { # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; cp $O/.cur.so $LIB; exit 1; }
  fault_guard $O/$name.log
  tail -1 $O/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); dg=d.get('diag_ms_per_step') or {}; print('$name', round(d['ms_per_step'],4), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']], 'phases', {k: round(v,4) for k,v in (d.get('phases_ms_per_step') or {}).items()}, 'trk', d.get('tracked_brackets'), 'clk', (d.get('gpu_diag') or {}).get('gfxclk_mhz_median'))"
}
for i in 1 2; do
  for v in tcol0 tcolpipe tcolw3; do
    cp tools/ablibs/$v.so $LIB
    b ${v}_cfg5_$i 300 --config cfg5 --steps 20 --warmup 3 --no-cpu --repeats 3
  done
  for v in tcol0 clsv; do
    cp tools/ablibs/$v.so $LIB
    b ${v}_cfg3_$i 300 --steps 20 --warmup 3 --no-cpu --repeats 3
    b ${v}_cfg2_$i 300 --config cfg2 --steps 20 --warmup 3 --no-cpu --repeats 3
  done
done
cp tools/ablibs/clsv.so $LIB
timeout -k 10 500 python -u -m pytest tests/test_gpu_collect.py tests/test_gpu_fullsize.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_clsv.log 2>&1; rc=$?
cp $O/.cur.so $LIB
echo "pytest clsv rc=$rc"; tail -1 $O/pytest_clsv.log; fault_guard $O/pytest_clsv.log
echo r4n done
