#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc csv output per kernel (mean per dispatch) and derive the conv
kernel's HBM traffic per launch (MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KB; on
gfx950 FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads -> x2)."""
import collections
import csv
import glob
import json
import os
import sys

out, tag = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for path in glob.glob(os.path.join(out, f"{tag}_pmc_*", "**", "*counter_collection*.csv"), recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "?")
            kname = "conv3x3_f32" if "conv3x3_f32_kernel" in name else (
                "conv3x3_smallc" if "smallc" in name else name.split("(")[0][-60:])
            vals[kname][row["Counter_Name"]].append((row.get("Dispatch_Id"), float(row["Counter_Value"])))
summary = {}
for k, cs in vals.items():
    summary[k] = {c: sum(v for _, v in xs) / max(1, len({d for d, _ in xs})) for c, xs in cs.items()}
    summary[k]["dispatches"] = max(len({d for d, _ in xs}) for xs in cs.values())
conv = summary.get("conv3x3_f32", {})
res = {"per_kernel_mean_per_dispatch": summary}
if "FETCH_SIZE" in conv and "WRITE_SIZE" in conv:
    fetch = conv["FETCH_SIZE"] * 1024
    write = conv["WRITE_SIZE"] * 1024
    res["conv_traffic"] = {"fetch_bytes_raw": fetch, "fetch_bytes_x2": 2 * fetch, "write_bytes": write,
                           "hbm_bytes_per_launch": 2 * fetch + write}
if "GRBM_GUI_ACTIVE" in conv:
    res["note"] = "GRBM_GUI_ACTIVE summed over 8 XCDs; effective clock = GRBM_GUI_ACTIVE/8/duration"
print(json.dumps(res, indent=1))
