"""Steady-state per-kernel durations from a rocprofv3 kernel trace: drops the
first `skip` calls of every kernel (warm-up launches run at a lower clock) and
prints calls, mean, median and min in ms.

Usage: python tools/ktimed.py <run_kernel_trace.csv> [skip]"""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
rows.sort(key=lambda r: int(r['Start_Timestamp']))
d = collections.defaultdict(list)
for r in rows:
    d[r['Kernel_Name']].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
out = []
for k, v in d.items():
    v = v[skip:] if len(v) > skip else v
    out.append((sum(v), k, len(v), statistics.mean(v), statistics.median(v), min(v)))
out.sort(reverse=True)
print(f"{'kernel':64s} {'calls':>5s} {'mean_ms':>9s} {'median_ms':>9s} {'min_ms':>9s}")
for tot, k, n, mean, med, mn in out:
    print(f"{k[:64]:64s} {n:5d} {mean:9.4f} {med:9.4f} {mn:9.4f}")
