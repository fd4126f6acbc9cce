# round 6, call l: SQ issue counters of k_pair_mcol (split build), two passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r6l
TAG=_r6l bash tools/pmc_sq.sh \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_sq_r6l/summary.csv gpurun_out/pmc_sq_r6l/p1 gpurun_out/pmc_sq_r6l/p2 && grep -i "mcol" gpurun_out/pmc_sq_r6l/summary.csv
# k_pair_mcol time under timing ablations (wrong results, timing only):
# abl1 = no band staging, abl2 = MFMAs only
cp svgdcpp_amd/libsvgdcpp_amd.so /tmp/r6l_cur.so
for v in split abl1 abl2; do
  cp tools/ablibs/$v.so svgdcpp_amd/libsvgdcpp_amd.so
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r6l/$v" -o run --output-format csv \
      -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/r6l/$v.log" 2>&1 ) || { echo "$v failed"; cp /tmp/r6l_cur.so svgdcpp_amd/libsvgdcpp_amd.so; exit 1; }
  python3 - "$v" <<'PY'
import csv,glob,sys
v=sys.argv[1]
for f in glob.glob(f"gpurun_out/r6l/{v}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mcol" in r["Name"] or "phi_sym" in r["Name"]:
            print(v, r["Name"][:40], r["Calls"], r["AverageNs"])
PY
done
cp /tmp/r6l_cur.so svgdcpp_amd/libsvgdcpp_amd.so
