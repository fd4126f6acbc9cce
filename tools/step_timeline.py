"""Print the kernel timeline (start offset, gap, duration) of the last full
step in a rocprofv3 kernel trace (steps start at k_mean_partial)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_mean_partial' in r['Kernel_Name']]
a, b = idx[-2], idx[-1]
t0 = int(rows[a]['Start_Timestamp'])
prev = None
for r in rows[a:b]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (s - prev) / 1e3 if prev else 0
    print(f"{(s - t0) / 1e3:9.1f} {gap:7.1f} {(e - s) / 1e3:8.1f}  {r['Kernel_Name'][:60]}")
    prev = e
print('step span us', (int(rows[b - 1]['End_Timestamp']) - t0) / 1e3)
