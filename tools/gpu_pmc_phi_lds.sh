#!/bin/bash
# LDS behaviour of the phi row stream at cfg3: waits for LDS data, bank
# conflicts, LDS-array activity (one counter pass), summarised per kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=_lds BENCH_ARGS="--repeats 1 --no-diag" bash tools/pmc_sq.sh "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE" || exit 1
python3 - gpurun_out/pmc_sq_lds/p1/run_counter_collection.csv <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in rows:
    k = r['Kernel_Name'][:60]
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    n[(k, r['Counter_Name'])] += 1
for k, c in acc.items():
    if 'phi_rows' not in k and 'mcol' not in k: continue
    disp = {m: c[m] / max(1, n[(k, m)]) for m in c}
    print(k)
    for m, v in sorted(disp.items()): print(f"   {m:24s} {v:.4g}")
PY
