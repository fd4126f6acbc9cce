"""Print a rocprofv3 kernel_stats.csv compactly: name, calls, total ms, avg ms, %."""
import csv
import sys

for x in csv.DictReader(open(sys.argv[1])):
    print(f"{x['Name'][:64]:64s} {x['Calls']:>5s} {float(x['TotalDurationNs'])/1e6:9.3f} "
          f"{float(x['AverageNs'])/1e6:8.4f} {x['Percentage'][:5]:>6s}")
