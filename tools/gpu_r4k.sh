#!/bin/bash
# k_phi_b3 variants (js-major Gram + truncating P split = default; 4-wave
# blocks; round-to-nearest P split): F32 suite on the default, then cfg5
# lines for each library build, interleaved on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4k
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_f32.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest.log; fault_guard $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
LIB=svgdcpp_amd/libsvgdcpp_amd.so
cp $LIB $O/.cur.so
for i in 1 2; do
  for v in b3pipe b3nw16; do
    cp tools/ablibs/$v.so $LIB
    timeout -k 10 300 python bench.py --config cfg5 --steps 20 --warmup 3 --no-cpu > $O/$v.$i.log 2>&1 || { echo "FAIL $v"; tail -5 $O/$v.$i.log; cp $O/.cur.so $LIB; exit 1; }
    fault_guard $O/$v.$i.log
    tail -1 $O/$v.$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); dg=d.get('diag_ms_per_step') or {}; print('$v', $i, round(d['ms_per_step'],4), 'phi', round(dg.get('phi_kernel'),4), 'clk', (d.get('gpu_diag') or {}).get('gfxclk_mhz_median'))"
  done
done
cp $O/.cur.so $LIB
echo r4k done
# HBM traffic of the two builds (FETCH_SIZE / WRITE_SIZE passes)
for v in b3pipe b3nw16; do
  cp tools/ablibs/$v.so $LIB
  TAG=_$v BENCH_ARGS="--config cfg5 --repeats 1 --no-diag" bash tools/pmc.sh FETCH_SIZE || { cp $O/.cur.so $LIB; exit 1; }
done
cp $O/.cur.so $LIB
echo r4k pmc done
