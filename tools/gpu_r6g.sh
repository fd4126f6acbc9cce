# round 6, call g: A/B of k_phi_b3 builds (tools/ablibs/il{0,3,4}.so: SVGD_B3_IL off / 3 / 4 VALU per
# MFMA) at cfg5 with RG 1 and 2, plus a bit-identity check of each build's phi against il0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
source tools/fault_guard.sh
mkdir -p gpurun_out/r6g
LIB=svgdcpp_amd/libsvgdcpp_amd.so
cp $LIB gpurun_out/r6g/.cur.so
chk() {
  timeout -k 10 120 python3 - "$1" <<'PY' || exit 1
import sys, hashlib, numpy as np, os
sys.path.insert(0, "oracle")
import oracle as O, svgdcpp_amd as S
from svgdcpp_amd import _capi as C
h = hashlib.sha256()
for rg in ("1", "2"):
    os.environ["SVGD_PHI_B3_RG"] = rg
    for n, d in ((3001, 64), (2049, 33), (4096, 48)):
        X = O.splitmix((n, d), 2.0, 7 * n + d); G = O.splitmix((n, d), 1.0, 7 * n + d + 1)
        c = S.Context(d, n, dtype=C.SVGD_F32); c.set_particles(X); ph = c.phi(G, 0.7 / d); c.close()
        h.update(ph.tobytes())
print(sys.argv[1], "phi sha", h.hexdigest()[:16])
PY
}
for v in il0 il3 il4; do cp tools/ablibs/$v.so $LIB; chk $v; done
for round in 1 2; do
  for v in il0 il3 il4; do
    cp tools/ablibs/$v.so $LIB
    for rg in 1 2; do
      SVGD_PHI_B3_RG=$rg timeout -k 10 300 python bench.py --config cfg5 --no-cpu --steps 20 --warmup 5 --repeats 3 > gpurun_out/r6g/$v.rg$rg.$round.log 2>&1 || { cp gpurun_out/r6g/.cur.so $LIB; exit 1; }
      fault_guard gpurun_out/r6g/$v.rg$rg.$round.log
      python3 -c "import json; d=json.loads(open('gpurun_out/r6g/$v.rg$rg.$round.log').read().strip().splitlines()[-1]); print('$v rg$rg', round(d['ms_per_step'],4), 'phi', round(d['diag_ms_per_step']['phi_kernel'],4), 'clk', d['gpu_timed'].get('gfxclk_mhz_median'), 'pw', d['gpu_timed'].get('power_w_median'))"
    done
  done
done
cp gpurun_out/r6g/.cur.so $LIB
