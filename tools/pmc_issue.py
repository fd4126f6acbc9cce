"""VALU issue evidence of the phi kernel from a tools/pmc_summary.py CSV.

Usage: python tools/pmc_issue.py <summary.csv> <kernel-substring> <pairs_per_launch> [n d world]

Writes profiles/phi_pmc_issue.json (read by bench.py as roofline.valu_issue_util
when kernel, source hash and workload match): VALU instructions per launch
and per pair-row (a wave64 instruction = one pair-row for 64 pairs, so per
pair-row = SQ_INSTS_VALU x 64 / pairs), and the issue utilisation
SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x GRBM_GUI_ACTIVE / 8).
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    path, kname, pairs = sys.argv[1], sys.argv[2], float(sys.argv[3])
    n, d, world = (int(x) for x in sys.argv[4:7]) if len(sys.argv) >= 7 else (65536, 8, 1)
    rows = [r for r in csv.DictReader(open(path)) if kname in r["kernel"]]
    if len(rows) != 1:
        sys.exit(f"kernel '{kname}' matched {len(rows)} rows")
    r = rows[0]
    valu = float(r["SQ_INSTS_VALU"])
    cycles = float(r["GRBM_GUI_ACTIVE"]) / 8
    sys.path.insert(0, ROOT)
    from bench import _kernel_src_sha

    rec = {"kernel": r["kernel"], "n": n, "d": d, "world": world, "src_sha16": _kernel_src_sha(),
           "valu_insts_per_launch": valu,
           "valu_insts_per_pair_row": valu * 64 / pairs,
           "valu_insts_per_simd_cycle": valu / (1024 * cycles),
           "valu_issue_util": valu * 4 / (1024 * cycles),
           "clock_ghz_under_load": float(r["clock_GHz"]) if r.get("clock_GHz") else None,
           "note": "fp64 VALU issues one wave64 instruction per 4 cycles per SIMD; util = insts x 4 / "
                   "(1024 SIMDs x cycles); clock = GRBM_GUI_ACTIVE/8/duration (counter run)",
           "source": os.path.relpath(path, ROOT)}
    with open(os.path.join(ROOT, "profiles", "phi_pmc_issue.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
