#!/usr/bin/env python3
"""Launch one conv3x3 configuration a few times on one layer shape (PMC / profiler driver).
python scripts/conv_one.py <cfg> [n cin h w cout up pad pool] [iters]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from arbitrarystyletransfer_amd import ops, synth  # noqa: E402

cfg = int(sys.argv[1])
shape = sys.argv[2:10] if len(sys.argv) >= 10 else ["16", "256", "128", "128", "256", "1", "zeros", "0"]
n, cin, h, w, cout, up = (int(v) for v in shape[:6])
pad, pool = shape[6], shape[7] == "1"
iters = int(sys.argv[10]) if len(sys.argv) > 10 else 3
dev = torch.device("cuda")
x = torch.from_numpy(synth.image(5, (n, cin, h, w))).to(dev)
wp = ops.pack_conv3x3(torch.from_numpy(synth.conv_weight(6, cout, cin, 3)).to(dev))
b = torch.from_numpy(synth.conv_bias(7, cout)).to(dev)
for _ in range(iters):
    ops.conv3x3(x, wp, b, cout, upsample=up, pad_mode=pad, want_pre=not pool, want_act=False, want_pool=pool, cfg=cfg)
torch.cuda.synchronize()
print("ok")
