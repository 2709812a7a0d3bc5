"""Summarise scripts/pmc_clock.sh: per kernel (name filter), the effective clock GRBM_GUI_ACTIVE / 8 /
duration (GRBM_GUI_ACTIVE is summed over the 8 XCDs; MI355X_MICROARCH.md 'DVFS give-back') and the MFMA
pipe busy fraction SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)."""
import collections
import csv
import glob
import os
import sys

d, filt = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
dur = {}
for f in kt:
    for r in csv.DictReader(open(f)):
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
ctr = collections.defaultdict(dict)
names = {}
for f in cc:
    for r in csv.DictReader(open(f)):
        if filt and filt not in r["Kernel_Name"]:
            continue
        ctr[r["Dispatch_Id"]][r["Counter_Name"]] = ctr[r["Dispatch_Id"]].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"].replace("(anonymous namespace)::", "").removeprefix("void ").split("(")[0][-70:]
rows = []
for did, c in ctr.items():
    t = dur.get(did)
    if not t or "GRBM_GUI_ACTIVE" not in c:
        continue
    cyc = c["GRBM_GUI_ACTIVE"] / 8
    rows.append((names[did], t, cyc / t / 1e9, c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * cyc)))
if not rows:
    print("no matching dispatches with both counters and durations")
    sys.exit(1)
tot = sum(r[1] for r in rows)
clk = sum(r[1] * r[2] for r in rows) / tot
mf = sum(r[1] * r[3] for r in rows) / tot
print(f"{len(rows)} dispatches matching '{filt}', {tot * 1e3:.2f} ms: time-weighted effective clock {clk:.3f} GHz, "
      f"MFMA busy {mf:.3f}")
by = collections.defaultdict(list)
for r in rows:
    by[r[0]].append(r)
for k, v in sorted(by.items(), key=lambda kv: -sum(r[1] for r in kv[1])):
    t = sum(r[1] for r in v)
    print(f"  {k}: {len(v)} dispatches {t * 1e3:.2f} ms clock {sum(r[1] * r[2] for r in v) / t:.3f} GHz "
          f"MFMA busy {sum(r[1] * r[3] for r in v) / t:.3f}")
