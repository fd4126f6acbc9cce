"""Per-kernel means of rocprofv3 --pmc counter passes (one CSV row per kernel).

Usage: python tools/pmc_summary.py <out.csv> <pass_dir> [<pass_dir> ...]

Each <pass_dir> holds a run_counter_collection.csv.  Counter values are summed
over the dimensions rocprofv3 reports for one dispatch, then averaged over the
dispatches of a kernel.  Derived columns (when their inputs are present):
  clock_GHz        = GRBM_GUI_ACTIVE / 8 (XCDs) / mean kernel duration
  valu_issue_frac  = SQ_ACTIVE_INST_VALU * 4 (quad-cycles) / (SQ_WAVE_CYCLES * 4)
                     -> share of wave lifetime spent issuing VALU
  valu_per_simd_cycle = SQ_INSTS_VALU / (1024 SIMDs * GRBM_GUI_ACTIVE / 8)
"""
import collections
import csv
import os
import sys


def load(path):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    names = {}
    for r in csv.DictReader(open(path)):
        key = (r["Kernel_Name"], r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        names[key] = r["Kernel_Name"]
    return per, dur


def main():
    out = sys.argv[1]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[2:]:
        per, dur = load(os.path.join(d, "run_counter_collection.csv"))
        for (k, _), cs in per.items():
            for c, v in cs.items():
                agg[k][c].append(v)
        for (k, _), t in dur.items():
            agg[k]["duration_s"].append(t)
    counters = sorted({c for k in agg for c in agg[k]})
    rows = []
    for k, cs in agg.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        if "GRBM_GUI_ACTIVE" in m and m.get("duration_s"):
            m["clock_GHz"] = m["GRBM_GUI_ACTIVE"] / 8 / m["duration_s"] / 1e9
            if "SQ_INSTS_VALU" in m:
                m["valu_per_simd_cycle"] = m["SQ_INSTS_VALU"] / (1024 * m["GRBM_GUI_ACTIVE"] / 8)
        if "SQ_ACTIVE_INST_VALU" in m and m.get("SQ_WAVE_CYCLES"):
            m["valu_issue_frac"] = m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"]
        rows.append((k, m))
    rows.sort(key=lambda r: -r[1].get("duration_s", 0))
    cols = counters + ["clock_GHz", "valu_per_simd_cycle", "valu_issue_frac"]
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel"] + cols)
        for k, m in rows:
            w.writerow([k[:90]] + [("%.6g" % m[c]) if c in m else "" for c in cols])
    for k, m in rows[:6]:
        print(k[:60], {c: round(m[c], 4) for c in cols if c in m})


if __name__ == "__main__":
    main()
