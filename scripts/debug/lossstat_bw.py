#!/usr/bin/env python3
"""Bandwidth of the loss-statistics launches of config 3 (style moments and the MVN-Huber content
loss; functional.mvn_huber / _style_terms) on the tap shapes of one AdaIN training step: median time
of 20 launches (HIP events) and the rate over the bytes they must read (x and y once per pass)."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from arbitrarystyletransfer_amd import functional as Fn  # noqa: E402
from arbitrarystyletransfer_amd._lib import lib, ptr  # noqa: E402


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


if __name__ == "__main__":
    for (n, c, s) in [(8, 64, 512), (8, 128, 256), (8, 256, 128), (8, 512, 64)]:
        x = torch.rand(n, c, s, s, device="cuda")
        y = torch.rand(n, c, s, s, device="cuda")
        nbytes = 2 * x.numel() * 4
        loss = Fn._acc(x)
        ps = torch.empty(n * c, 6, device="cuda")
        t_m = timed(lambda: Fn.mvn_huber(x, y, 1.0, loss, ps))
        planes, hw = n * c, s * s
        ws = Fn.workspace(lib().ast_plane_stats_workspace_floats(planes, hw), x.device)
        st = torch.empty(planes, 4, device="cuda")
        ra = torch.empty(planes, device="cuda")
        rb = torch.empty(planes, device="cuda")
        t_s = timed(lambda: lib().ast_style_moments_ws_f32(ptr(x), ptr(y), planes, hw, 1.0, None, ptr(st), ptr(loss),
                                                           ptr(ra), ptr(rb), ptr(ws), ws.numel(), Fn._s(x)))
        dx = torch.empty_like(x)
        Fn.mvn_huber(x, y, 1.0, loss, ps)
        t_b = timed(lambda: lib().ast_mvn_huber_backward_f32(ptr(x), ptr(y), ptr(ps), planes, hw, 1.0, None, ptr(dx), 0,
                                                              Fn._s(x)))
        print(f"  mvn_huber_backward {t_b * 1e3:7.1f} us ({3 * x.numel() * 4 / t_b / 1e6:5.0f} GB/s)", flush=True)
        dG = torch.rand(n, c, c, device="cuda")
        raa = torch.rand(planes, device="cuda")
        rbb = torch.rand(planes, device="cuda")
        t_gb = timed(lambda: lib().ast_gram_backward_f32(ptr(x), ptr(dG), ptr(dx), ptr(raa), ptr(rbb), n, c, hw,
                                                          1.0 / (c * hw), None, 0, Fn._s(x)))
        print(f"  gram_backward {t_gb * 1e3:7.1f} us ({2 * c * c * hw * n * 2 / t_gb / 1e9:5.0f} TF, "
              f"{3 * x.numel() * 4 / t_gb / 1e6:5.0f} GB/s over F read twice + dF)", flush=True)
        gx = torch.empty(n, c, c, device="cuda")
        t_g = timed(lambda: Fn.gram(x, gx, 1.0 / (c * hw)))
        print(f"{n}x{c}x{s}^2: mvn_huber {t_m * 1e3:7.1f} us ({2 * nbytes / t_m / 1e6:5.0f} GB/s over 2 passes)   "
              f"style_moments {t_s * 1e3:7.1f} us ({nbytes / t_s / 1e6:5.0f} GB/s)   gram(x) {t_g * 1e3:7.1f} us "
              f"({nbytes / 2 / t_g / 1e6:5.0f} GB/s)", flush=True)
