"""Per-launch breakdown of one config-5 step (MobileNet variant, bf16, B=32, 1024^2): every
expand_dw / pw / dense launch with its time, algorithmic GB/s and depthwise FMA rate.
python scripts/mb_launch_breakdown.py [batch] [size]"""
import json
import os
import re
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbitrarystyletransfer_amd import models, ops, synth  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    net = models.AST(exporting=True).load_live_init().eval().to(dev).to(bf)
    c = torch.from_numpy(synth.image(821, (B, 3, S, S))).to(dev).to(bf)
    s = torch.from_numpy(synth.image(822, (B, 3, S, S))).to(dev).to(bf)
    with torch.no_grad():
        for _ in range(2):
            net(c, s)
        torch.cuda.synchronize()
        timer = ops.LaunchTimer()
        with timer:
            net(c, s)
        torch.cuda.synchronize()
    rows, tot = [], 0.0
    for tag, nb, ms in timer.results():
        tot += ms
        row = {"tag": tag, "ms": round(ms, 3), "gbs": round(-nb / ms / 1e6, 1)}
        m = re.match(r"mb expand_dw k(\d)s(\d)( up)? (\d+)->(\d+) (\d+)x(\d+)", tag)
        if m:
            k, st, up, cin, hid, ho, wo = m.groups()
            k, cin, hid, ho, wo = int(k), int(cin), int(hid), int(ho), int(wo)
            n = B if "expand_dw" in tag else B
            dw = 2 * n * hid * ho * wo * k * k
            row["dw_tflops"] = round(dw / ms / 1e9, 2)
        rows.append(row)
    rows_sorted = sorted(rows, key=lambda r: -r["ms"])
    for r in rows_sorted:
        print(json.dumps(r))
    print(json.dumps({"total_ms": round(tot, 2)}))
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/mb_launches.json", "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
