#!/bin/bash
# k_phi_b3 wave stagger (waves 4-7 VALU-first, SVGD_B3_STAGGER) and the
# 4-waves/SIMD bound, vs the previous build (head): F32 suite on the default,
# then interleaved cfg5 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
source tools/fault_guard.sh
O=gpurun_out/r4v
mkdir -p $O
LIB=svgdcpp_amd/libsvgdcpp_amd.so
cp $LIB $O/.cur.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_f32.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest.log; fault_guard $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for i in 1 2; do
  for v in head b3st0 b3st1; do
    cp tools/ablibs/$v.so $LIB
    timeout -k 10 300 python bench.py --config cfg5 --steps 20 --warmup 3 --no-cpu --repeats 3 > $O/$v.$i.log 2>&1 || { echo "FAIL $v"; tail -5 $O/$v.$i.log; cp $O/.cur.so $LIB; exit 1; }
    fault_guard $O/$v.$i.log
    tail -1 $O/$v.$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); dg=d['diag_ms_per_step']; print('$v', $i, round(d['ms_per_step'],4), 'runs', [round(x,3) for x in d['repeats']['ms_per_step']], 'phi', round(dg['phi_kernel'],4), 'clk', d['gpu_timed'].get('gfxclk_mhz_median'))"
  done
done
cp $O/.cur.so $LIB
echo r4v done
