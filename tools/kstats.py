"""Print a rocprofv3 kernel_stats.csv (or the newest one under a directory) as a table."""
import csv
import glob
import os
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
if os.path.isdir(path):
    path = max(glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True),
               key=os.path.getmtime)
print(path)
for r in csv.DictReader(open(path)):
    print(f"{r['Name'][:64]:64s} calls={r['Calls']:>4} avg_ms={float(r['AverageNs']) / 1e6:9.3f} "
          f"pct={float(r['Percentage']):6.2f}")
