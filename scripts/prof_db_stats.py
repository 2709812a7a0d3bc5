"""Kernel statistics from a rocprofv3 results database (run_results.db; this rocprofv3 writes the
database instead of the --stats CSV): writes <out>.csv in the kernel_stats.csv layout (Name, Calls,
TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, StdDev) and prints per-grid rows for the
kernels whose names contain the given substrings.
usage: prof_db_stats.py run_results.db out.csv [substr ...]"""
import csv
import math
import sqlite3
import sys
from collections import defaultdict

db, out, subs = sys.argv[1], sys.argv[2], sys.argv[3:]
c = sqlite3.connect(db)
rows = list(c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x from kernels"))
by = defaultdict(list)
for n, d, *_ in rows:
    by[n].append(float(d))
tot = sum(sum(v) for v in by.values())
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for n, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        m = sum(v) / len(v)
        sd = math.sqrt(sum((x - m) ** 2 for x in v) / len(v))
        w.writerow([n, len(v), sum(v), m, 100.0 * sum(v) / tot, min(v), max(v), sd])
grid = defaultdict(list)
for n, d, gx, gy, gz, wx in rows:
    if any(s in n for s in subs):
        grid[(n.replace("(anonymous namespace)::", "").split("(")[0][-40:], gx // max(wx, 1), gy, gz)].append(float(d))
for k, v in sorted(grid.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v) / 1e6:9.3f} ms {len(v):5d}x {sum(v) / len(v) / 1e3:9.1f} us  {k}")
