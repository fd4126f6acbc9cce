"""Print the kernel timeline (start offset, gap, duration) of one step of a
rocprofv3 kernel trace (steps start at the centring): the middle step of
the trace, which lies in bench.py's timed repeats (the diagnostic pass with
its extra events comes after them).  Also prints the median step span over
all steps.  With a second argument (the run's memory-copy trace CSV) the
copies that start inside the step are listed too, marked 'copy'."""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# a step starts at its centring (k_center / k_center_d), or at the
# k_mean_partial right before it (steps whose mean partials the previous
# update epilogue did not leave)
idx = [i - 1 if i > 0 and 'k_mean_partial' in rows[i - 1]['Kernel_Name'] else i
       for i, r in enumerate(rows) if 'k_center' in r['Kernel_Name']]
spans = [(int(rows[j - 1]['End_Timestamp']) - int(rows[i]['Start_Timestamp'])) / 1e3
         for i, j in zip(idx, idx[1:])]
m = (len(idx) - 1) // 2
a, b = idx[m], idx[m + 1]
t0 = int(rows[a]['Start_Timestamp'])
t1 = int(rows[b]['Start_Timestamp'])
print(f"step {m} of {len(idx) - 1} (middle of the trace)")
prev = None
for r in rows[a:b]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (s - prev) / 1e3 if prev else 0
    print(f"{(s - t0) / 1e3:9.1f} {gap:7.1f} {(e - s) / 1e3:8.1f}  {r['Kernel_Name'][:60]}")
    prev = e
print('step span us', (int(rows[b - 1]['End_Timestamp']) - t0) / 1e3,
      'median over steps', round(statistics.median(spans), 3) if spans else None)
if len(sys.argv) > 2:
    for r in sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r['Start_Timestamp'])):
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        if t0 - 200000 <= s < t1:
            what = r.get('Direction') or r.get('Operation') or ''
            print(f"{(s - t0) / 1e3:9.1f} {'copy':>7} {(e - s) / 1e3:8.1f}  {what} {r.get('Size', r.get('Bytes', ''))}")
