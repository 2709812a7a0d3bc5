"""Top kernels by total time from a rocprofv3 --stats output directory (any *kernel_stats.csv
below it): python scripts/kernel_stats_top.py DIR [N]"""
import csv
import glob
import os
import sys

d, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12
files = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
if not files:
    sys.exit(f"no kernel_stats.csv under {d}")
rows = []
for f in files:
    with open(f) as fh:
        rows += list(csv.DictReader(fh))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"  total {tot / 1e6:.2f} ms over {sum(int(r['Calls']) for r in rows)} dispatches")
for r in rows[:n]:
    name = r["Name"].replace("(anonymous namespace)::", "")
    name = name.split("(")[0] if not name.startswith("void ") else name[5:].split("(")[0]
    print(f"  {float(r['TotalDurationNs']) / 1e6:9.3f} ms {int(r['Calls']):5d}x {float(r['AverageNs']) / 1e3:9.1f} us  {name[-70:]}")
