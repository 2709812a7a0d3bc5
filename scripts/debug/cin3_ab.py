#!/usr/bin/env python3
"""A/B of the 1..3-channel-input convs: the direct VALU kernel (cfg 22) against the split-bf16 MFMA
kernel (cfg 42: 16-row tiles, 43: 8-row tiles), on the launches of configs 2 / 3 and the 160^2
trainers. Prints per shape and configuration the median time (HIP events, 20 launches), the output
bandwidth, and the largest error against a float64 CPU conv of image 0 (relative to max |ref|).
Usage: python3 scripts/debug/cin3_ab.py [cfg,cfg,...]
"""
import os
import statistics
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from arbitrarystyletransfer_amd import ops  # noqa: E402
from arbitrarystyletransfer_amd._lib import check, lib, ptr, stream_ptr  # noqa: E402
from arbitrarystyletransfer_amd.functional import _TF  # noqa: E402

CFGS = [int(c) for c in sys.argv[1].split(",")] if len(sys.argv) > 1 else [22, 42, 43]
MEAN = torch.tensor([0.485, 0.456, 0.406])
STD = torch.tensor([0.229, 0.224, 0.225])


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


def ref_fwd(x, w, b, norm, pad):
    x = x[:1].double().cpu()
    if norm:
        x = (x - MEAN.double().view(1, 3, 1, 1)) / STD.double().view(1, 3, 1, 1)
    x = F.pad(x, (1, 1, 1, 1), mode="reflect" if pad == "reflect" else "constant")
    return F.conv2d(x, w.double().cpu(), b.double().cpu())


def fwd_case(n, s, cout, norm, pad, pre, act):
    g = torch.Generator().manual_seed(n * 7 + s + cout)
    x = torch.rand(n, 3, s, s, generator=g).cuda()
    w = (torch.randn(cout, 3, 3, 3, generator=g) * 0.2).cuda()
    b = (torch.randn(cout, generator=g) * 0.1).cuda()
    wp = ops.pack_conv3x3(w)
    mean, std = (MEAN.cuda(), STD.cuda()) if norm else (None, None)
    ref = ref_fwd(x, w, b, norm, pad)
    out_bytes = n * cout * s * s * 4 * (int(pre) + int(act))
    print(f"fwd {n}x3x{s}^2->{cout} {'norm ' if norm else ''}{pad} pre={int(pre)} act={int(act)}")
    for cfg in CFGS:
        run = lambda: ops.conv3x3(x, wp, b, cout, pad_mode=pad, in_mean=mean, in_std=std,  # noqa: E731
                                  want_pre=pre, want_act=act, cfg=cfg)
        try:
            p, a, _ = run()
        except Exception as e:  # unsupported configuration
            print(f"  cfg {cfg}: {e}")
            continue
        ms = timed(run)
        err = 0.0
        if p is not None:
            err = max(err, ((p[:1].double().cpu() - ref).abs().max() / ref.abs().max()).item())
        if a is not None:
            err = max(err, ((a[:1].double().cpu() - ref.clamp_min(0)).abs().max() / ref.abs().max()).item())
        print(f"  cfg {cfg}: {ms * 1e3:8.1f} us  {out_bytes / ms / 1e6:7.0f} GB/s  rel_err {err:.2e}")


def dgrad_case(n, s, cin):
    """input gradient of a cin -> 3 conv: a 3-channel same conv of dy, ReLU mask of its input"""
    g = torch.Generator().manual_seed(n + s)
    dy = torch.randn(n, 3, s, s, generator=g).cuda()
    w = (torch.randn(3, cin, 3, 3, generator=g) * 0.1).cuda()
    mask = torch.randn(n, cin, s, s, generator=g).cuda().clamp_min(0)
    wtf = _TF.get(w, None)
    d0 = dy[:1].double().cpu()
    ref = F.conv_transpose2d(d0, w.double().cpu(), padding=1)
    ref = torch.where(mask[:1].double().cpu() > 0, ref, torch.zeros_like(ref))
    out_bytes = n * cin * s * s * 4 * 2  # dx written, mask read
    print(f"dgrad {n}x3x{s}^2 -> dx {cin} ch (mask)")
    for cfg in CFGS:
        dx = torch.empty(n, cin, s, s, device="cuda")
        run = lambda: lib().ast_conv3x3_dgrad_f32(cfg, ptr(dy), ptr(wtf), ptr(dx), ptr(mask), None, None,  # noqa: E731
                                                  n, 3, s, s, cin, 1, stream_ptr(dy.device))
        rc = run()
        if rc != 0:
            print(f"  cfg {cfg}: rc {rc}")
            continue
        ms = timed(run)
        err = ((dx[:1].double().cpu() - ref).abs().max() / ref.abs().max()).item()
        print(f"  cfg {cfg}: {ms * 1e3:8.1f} us  {out_bytes / ms / 1e6:7.0f} GB/s  rel_err {err:.2e}")


if __name__ == "__main__":
    torch.backends.cudnn.allow_tf32 = False
    fwd_case(16, 512, 64, True, "zeros", False, True)   # config 2 conv_1 (content + style)
    fwd_case(16, 512, 64, True, "zeros", True, True)    # config 3 loss network conv_1
    fwd_case(16, 160, 64, True, "zeros", True, True)    # 160^2 trainers' loss network
    fwd_case(16, 160, 16, False, "reflect", False, True)  # 3 -> 16 reflect (AST transformer stem)
    fwd_case(3, 100, 40, False, "zeros", True, True)    # ragged: W % 64, H % 16, cout % 16
    fwd_case(2, 66, 130, True, "reflect", True, False)  # two cout groups
    dgrad_case(8, 512, 64)                               # config 3 decoder's last conv
    dgrad_case(16, 160, 64)
