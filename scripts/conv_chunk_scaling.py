#!/usr/bin/env python3
"""Per-launch fixed cost of the conv kernel: one layer shape at Cin = 16..512 (1..32 K-chunks),
tuned configuration, HIP-event median of 7. time(Cin) = fixed + chunks * per_chunk."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from arbitrarystyletransfer_amd import ops, synth  # noqa: E402

dev = torch.device("cuda:0")
n, h, w, cout = int(sys.argv[1]) if len(sys.argv) > 1 else 16, 128, 128, 256
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 24
pts = []
for cin in (16, 32, 64, 128, 256, 512):
    x = torch.from_numpy(synth.image(5, (n, cin, h, w))).to(dev)
    wp = ops.pack_conv3x3(torch.from_numpy(synth.conv_weight(6, cout, cin, 3)).to(dev))
    b = torch.zeros(cout, device=dev)
    f = lambda: ops.conv3x3(x, wp, b, cout, want_pre=False, want_act=True, cfg=cfg)  # noqa: E731
    for _ in range(2):
        f()
    ts = []
    for _ in range(7):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        f()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    t = statistics.median(ts)
    pts.append((cin // 16, t))
    print(f"cin {cin:4d} chunks {cin // 16:3d}: {t:.4f} ms", flush=True)
k = [c for c, _ in pts]
t = [v for _, v in pts]
mk, mt = sum(k) / len(k), sum(t) / len(t)
slope = sum((a - mk) * (b - mt) for a, b in zip(k, t)) / sum((a - mk) ** 2 for a in k)
print(f"fit: fixed {mt - slope * mk:.4f} ms + {slope:.4f} ms per chunk")
