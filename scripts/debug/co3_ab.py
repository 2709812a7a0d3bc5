#!/usr/bin/env python3
"""A/B of the Cout <= 3 convs: the direct VALU kernels (cfg 10, 36) against the split-bf16 MFMA
kernel with the taps on the M side (cfg 44, round 6: measured here and removed, see DESIGN.md
conv3x3_smallc_kernel), on the launches of configs 2 / 3 and the 160^2 trainers: median time of 20
launches (HIP events) and the error against a float64 CPU conv of image 0."""
import os
import statistics
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from arbitrarystyletransfer_amd import ops  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


for (n, cin, h, w, cout, pad, pre, act) in [(8, 64, 512, 512, 3, "reflect", True, False),
                                           (16, 64, 512, 512, 3, "zeros", True, False),
                                           (8, 64, 160, 160, 3, "reflect", True, False),
                                           (8, 16, 160, 160, 3, "reflect", False, True),
                                           (2, 40, 37, 150, 2, "zeros", True, True)]:
    g = torch.Generator().manual_seed(n + cin + h)
    x = torch.rand(n, cin, h, w, generator=g).cuda()
    wt = (torch.randn(cout, cin, 3, 3, generator=g) * 0.05).cuda()
    b = (torch.randn(cout, generator=g) * 0.1).cuda()
    wp = ops.pack_conv3x3(wt)
    ref = F.conv2d(F.pad(x[:1].double().cpu(), (1, 1, 1, 1), mode="reflect" if pad == "reflect" else "constant"),
                   wt.double().cpu(), b.double().cpu())
    print(f"{n}x{cin}x{h}x{w}->{cout} {pad}", flush=True)
    for cfg in (10, 36, 44):
        run = lambda: ops.conv3x3(x, wp, b, cout, pad_mode=pad, want_pre=pre, want_act=act, cfg=cfg)  # noqa: E731
        try:
            p, a, _ = run()
        except Exception as e:
            print(f"  cfg {cfg}: {e}")
            continue
        ms = timed(run)
        o = p if p is not None else a
        r = ref if p is not None else ref.clamp_min(0)
        err = float((o[:1].double().cpu() - r).abs().max() / r.abs().max())
        print(f"  cfg {cfg}: {ms * 1e3:8.1f} us  {x.numel() * 4 / ms / 1e6:6.0f} GB/s of x  rel_err {err:.2e}", flush=True)
