#!/bin/bash
# k_pair_mcol time per library variant (tools/ablibs/<v>.so in place of the
# library, rocprofv3 kernel trace of a short cfg3 bench): A/B of collect
# builds and the timing ablations of SVGD_MCOL_ABL (whose results are wrong:
# their runs only time the kernel).  Usage: bash tools/gpu_mcol_abl.sh base il abl1 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=$REPO/gpurun_out/abl
mkdir -p $OUT
source tools/fault_guard.sh
LIB=svgdcpp_amd/libsvgdcpp_amd.so
cp $LIB $OUT/.cur.so
for round in $(seq ${ROUNDS:-1}); do
  for v in "$@"; do
    cp tools/ablibs/$v.so $LIB
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/$v.$round -o run --output-format csv \
       -- python3 $REPO/bench.py --config ${CFG:-cfg3} --steps 6 --warmup 2 --repeats 1 --no-cpu --no-diag > $OUT/$v.$round.log 2>&1)
    rc=$?
    fault_guard $OUT/$v.$round.log
    case $rc in 124|134|137|139) echo "$v: rc=$rc, stopping"; cp $OUT/.cur.so $LIB; exit $rc;; esac
    python3 - $v $rc $OUT/$v.$round/run_kernel_trace.csv <<'PY'
import csv, sys, statistics
v, rc, path = sys.argv[1:4]
try:
    rows = list(csv.DictReader(open(path)))
except OSError:
    print(v, "rc", rc, "no trace"); sys.exit(0)
m = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows if 'k_pair_mcol' in r['Kernel_Name']]
phi = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows if 'k_phi_rows' in r['Kernel_Name']]
if m:
    print(f"{v:8s} rc {rc} mcol n {len(m)} median {statistics.median(m[2:] or m):.1f} min {min(m):.1f} us; phi median {statistics.median(phi) if phi else 0:.1f}")
else:
    print(v, "rc", rc, "no mcol launches")
PY
  done
done
cp $OUT/.cur.so $LIB
exit 0
