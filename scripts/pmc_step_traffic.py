"""Whole-step HBM traffic from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (scripts/measure_profiles.sh
layout: gpurun_out/<tag>_pmc_*/.../*counter_collection.csv): every dispatch of the run summed, FETCH_SIZE
doubled (MI355X_MICROARCH.md gfx950 correction), divided by the steps the run made, counted as the
dispatches of a kernel that runs a known number of times per step.
python scripts/pmc_step_traffic.py <tag> <per-step-kernel-substring> <launches-per-step> [out.json]"""
import collections
import csv
import glob
import json
import os
import sys

tag, marker, per = sys.argv[1], sys.argv[2], int(sys.argv[3])
root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
tot, fam, marks = collections.Counter(), collections.Counter(), collections.Counter()
for f in sorted(glob.glob(os.path.join(root, f"{tag}_pmc_*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        ctr, v, name = r["Counter_Name"], float(r["Counter_Value"]) * 1024.0, r["Kernel_Name"]
        b = 2 * v if ctr == "FETCH_SIZE" else v
        tot[ctr] += b
        key = name.replace("void ", "").replace("(anonymous namespace)::", "").replace("ast_mb::", "")
        key = key.split("(")[0]
        fam[key] += b
        if marker in name:
            marks[ctr] += 1
steps = marks["FETCH_SIZE"] / per
res = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ({tag}), all dispatches, FETCH_SIZE x2; "
                 f"steps = '{marker}' dispatches / {per}",
       "steps": steps, "fetch_x2_gb_per_step": tot["FETCH_SIZE"] / steps / 1e9,
       "write_gb_per_step": tot["WRITE_SIZE"] / steps / 1e9,
       "hbm_gb_per_step": (tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) / steps / 1e9,
       "by_kernel_gb_per_step": {k: round(v / steps / 1e9, 3) for k, v in fam.most_common(20)}}
print(json.dumps(res, indent=1))
if len(sys.argv) > 4:
    with open(sys.argv[4], "w") as f:
        json.dump(res, f, indent=1)
