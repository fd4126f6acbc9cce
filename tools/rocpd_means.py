"""Per-kernel dispatch count, mean and median duration (us) from a rocprofv3
SQLite output (run_results.db), for kernels whose name matches a regex.
Usage: python3 tools/rocpd_means.py <db> [regex]"""
import collections
import re
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
dur = collections.defaultdict(list)
for row in db.execute("select * from kernels"):
    r = dict(zip(cols, row))
    name = r.get("name") or r.get("kernel_name") or ""
    if pat.search(name):
        dur[name].append((r["end"] - r["start"]) / 1e3)
print("==", sys.argv[1])
for name, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    s = sorted(v)
    print(f"{len(v):6d}  mean {sum(v) / len(v):10.2f}  median {s[len(s) // 2]:10.2f}  {name[:90]}")
