#!/usr/bin/env python3
"""Time the Cout <= 3 weight gradients (functional.conv_weight_grad) of the trainers: the config-3
decoder's 64 -> 3 conv and the 160^2 image convs. Run with AST_WGRAD_CO3=0 (VALU wgrad_smallco) and
=1 (split-bf16 MFMA, wgrad_co3.hip); prints median ms of 20 (HIP events) and the error against a
float64 CPU weight gradient of image 0."""
import os
import statistics
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from arbitrarystyletransfer_amd import functional as Fn  # noqa: E402


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


tag = os.environ.get("AST_WGRAD_CO3", "1")
for (n, cin, s, cout, pad) in [(8, 64, 512, 3, "reflect"), (16, 64, 160, 3, "reflect"), (8, 16, 160, 3, "reflect")]:
    x = torch.rand(n, cin, s, s, device="cuda")
    dy = torch.rand(n, cout, s, s, device="cuda") * 2 - 1
    ms = timed(lambda: Fn.conv_weight_grad(x, dy, cout, 1, pad))
    dw, db = Fn.conv_weight_grad(x[:1], dy[:1], cout, 1, pad)
    xc = F.pad(x[:1].double().cpu(), (1, 1, 1, 1), mode=pad if pad == "reflect" else "constant")
    ref = torch.nn.grad.conv2d_weight(xc, (cout, cin, 3, 3), dy[:1].double().cpu())
    err = float((dw.double().cpu() - ref).abs().max() / ref.abs().max())
    print(f"co3={tag} {n}x{cin}x{s}^2->{cout} {pad}: {ms * 1e3:8.1f} us  ({n * cin * s * s * 4 / ms / 1e6:5.0f} GB/s of x)"
          f"  rel_err {err:.2e}", flush=True)
