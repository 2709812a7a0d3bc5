"""Summarise a rocprofv3 kernel trace per (kernel, grid): ms per step (steps = adam_kernel launches)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2] if len(sys.argv) > 2 else ""
steps = max(1, sum(1 for r in rows if "adam_kernel" in r["Kernel_Name"]))
agg = collections.defaultdict(lambda: [0, 0.0])
fam = collections.defaultdict(float)
for r in rows:
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").replace("ast_det::", "").split("(")[0]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    fam[n.split("<")[0]] += d
    if pat not in n:
        continue
    key = (n[:64], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), r["Grid_Size_Y"], r["Grid_Size_Z"])
    agg[key][0] += 1
    agg[key][1] += d
print(f"steps {steps}, total {sum(fam.values()) / steps / 1e3:.2f} ms/step")
for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:30]:
    print(f"  {v / steps / 1e3:7.3f} ms/step  {k}")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    print(f"{v[1] / steps / 1e3:7.3f} ms/step {v[0] / steps:5.1f}x {v[1] / v[0]:8.1f}us {k}")
