"""HBM traffic per dispatch of a kernel family from rocprofv3 FETCH_SIZE / WRITE_SIZE passes
(scripts/pmc_kernel.sh layout: gpurun_out/<tag>_pmc_*/.../*counter_collection.csv).
FETCH_SIZE is doubled per MI355X_MICROARCH.md's gfx950 correction; both counters are in KB.
python scripts/pmc_traffic.py <tag> <kernel-substring> [out.json] [exclude-substring]
PMC_COMMIT=<sha> names the tree the box ran (default: this checkout's HEAD, +uncommitted if dirty)."""
import collections
import csv
import glob
import json
import os
import sys

tag, filt = sys.argv[1], sys.argv[2]
excl = sys.argv[4] if len(sys.argv) > 4 else None
root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
tot, n = collections.Counter(), collections.Counter()
for f in sorted(glob.glob(os.path.join(root, f"{tag}_pmc_*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        if filt in r["Kernel_Name"] and not (excl and excl in r["Kernel_Name"]):
            tot[r["Counter_Name"]] += float(r["Counter_Value"]) * 1024.0
            n[r["Counter_Name"]] += 1
fetch = tot["FETCH_SIZE"] / max(n["FETCH_SIZE"], 1)
write = tot["WRITE_SIZE"] / max(n["WRITE_SIZE"], 1)
import subprocess
try:
    sha = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True,
                         cwd=os.path.dirname(root)).stdout.strip()
    dirty = subprocess.run(["git", "status", "--porcelain", "--untracked-files=no"], capture_output=True,
                           text=True, cwd=os.path.dirname(root)).stdout.strip()
    commit = os.environ.get("PMC_COMMIT") or sha + ("+uncommitted" if dirty else "")
except OSError:
    commit = "unknown"
excl_txt = f" (not '{excl}')" if excl else ""
res = {"commit": commit, "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ({tag}); mean per '{filt}'{excl_txt} dispatch over "
                 f"{n['FETCH_SIZE']} dispatches; FETCH_SIZE x2 per MI355X_MICROARCH.md gfx950 correction",
       "fetch_bytes_raw": fetch, "fetch_bytes_x2": 2 * fetch, "write_bytes": write,
       "hbm_bytes_per_launch": 2 * fetch + write}
print(json.dumps(res, indent=1))
if len(sys.argv) > 3:
    with open(sys.argv[3], "w") as f:
        json.dump(res, f, indent=1)
