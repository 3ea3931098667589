"""Print the per-kernel average durations of a rocprofv3 --stats output directory."""
import csv
import glob
import sys

paths = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)
if not paths:
    sys.exit(f"no kernel_stats.csv under {sys.argv[1]}")
with open(paths[0]) as f:
    rows = list(csv.DictReader(f))
for r in rows[:16]:
    name = r["Name"].split("(")[0].replace("void admm::", "")
    print(f"{float(r['AverageNs']) / 1e3:8.2f} us x{int(r['Calls']):5d} {float(r['Percentage']):6.2f}%  {name}")
