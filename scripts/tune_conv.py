#!/usr/bin/env python3
"""Sweep every conv3x3 kernel configuration over the layer shapes of the benchmarked path and
write the fastest per shape to arbitrarystyletransfer_amd/conv_tuning.json (read by ops.conv3x3).

Each (shape, config) is timed with HIP events on the launch stream: 2 warm-up launches, then the
median of 5. Configurations a shape does not support are rejected on the host (no launch).
"""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from arbitrarystyletransfer_amd import ops, synth  # noqa: E402
from arbitrarystyletransfer_amd._lib import lib  # noqa: E402

# (n, cin, h_in, w_in, cout, up, pad, pool) of the bench step (config 2, B=8 -> encoder sees 16)
ENC = [(3, 64, 512, False), (64, 64, 512, True), (64, 128, 256, False), (128, 128, 256, True),
       (128, 256, 128, False), (256, 256, 128, False), (256, 256, 128, False), (256, 256, 128, True),
       (256, 512, 64, False)]
DEC = [(512, 256, 64, 1), (256, 256, 64, 2), (256, 256, 128, 1), (256, 256, 128, 1), (256, 128, 128, 1),
       (128, 128, 128, 2), (128, 64, 256, 1), (64, 64, 256, 2), (64, 3, 512, 1)]


def shapes(batch):
    out = []
    for cin, cout, s, pool in ENC:
        out.append((2 * batch, cin, s, s, cout, 1, "zeros", pool))
    for cin, cout, s, up in DEC:
        out.append((batch, cin, s, s, cout, up, "reflect", False))
    return out


def ae_shapes(batch=16, size=160):
    """The conv3x3 launches of one AutoEncoder training step (bench.py --mode ae-train: the VGG
    loss network's forward passes and input-gradient convs), captured from a live step."""
    from arbitrarystyletransfer_amd import models
    from arbitrarystyletransfer_amd.train import AutoencoderTrainer, default_ae_args
    seen = []
    orig = ops.conv3x3

    def spy(x, w_packed, bias, cout, *, upsample=1, pad_mode="zeros", want_pool=False, x2=None, **kw):
        n = int(x.shape[0]) + (int(x2.shape[0]) if x2 is not None else 0)
        shp = (n, int(x.shape[1]), int(x.shape[2]), int(x.shape[3]), cout, upsample, pad_mode, want_pool)
        if shp not in seen:
            seen.append(shp)
        return orig(x, w_packed, bias, cout, upsample=upsample, pad_mode=pad_mode, want_pool=want_pool, x2=x2, **kw)

    ops.conv3x3 = spy
    try:
        tr = AutoencoderTrainer(default_ae_args(batch_size=batch), device="cuda",
                                model=models.AutoEncoder().load_live_init())
        tr.train_step(torch.from_numpy(synth.image(901, (batch, 3, size, size))).cuda(), record=False)
        torch.cuda.synchronize()
    finally:
        ops.conv3x3 = orig
    return seen


def adain_train_shapes(batch=16, size=512):
    """The conv3x3 launches of one AdaIN training step (bench.py --mode train, config 3: decoder,
    loss network, their input-gradient convs), captured from a live step."""
    from arbitrarystyletransfer_amd.train import AdaINTrainer, default_args
    seen = []
    orig = ops.conv3x3

    def spy(x, w_packed, bias, cout, *, upsample=1, pad_mode="zeros", want_pool=False, x2=None, **kw):
        n = int(x.shape[0]) + (int(x2.shape[0]) if x2 is not None else 0)
        shp = (n, int(x.shape[1]), int(x.shape[2]), int(x.shape[3]), cout, upsample, pad_mode, want_pool)
        if shp not in seen:
            seen.append(shp)
        return orig(x, w_packed, bias, cout, upsample=upsample, pad_mode=pad_mode, want_pool=want_pool, x2=x2, **kw)

    ops.conv3x3 = spy
    try:
        tr = AdaINTrainer(default_args(batch_size=batch), device="cuda")
        c = torch.from_numpy(synth.image(903, (batch, 3, size, size))).cuda()
        s = torch.from_numpy(synth.image(904, (batch, 3, size, size))).cuda()
        tr.train_step(c, s, record=False)
        torch.cuda.synchronize()
    finally:
        ops.conv3x3 = orig
    return seen


def ast_shapes(batch=8, size=160):
    """The conv3x3 launches of one ASTTrainer step (bench.py --mode ast-train: the loss network's
    passes over the packed small planes and their input-gradient convs, the image convs)."""
    from arbitrarystyletransfer_amd import models
    from arbitrarystyletransfer_amd.train import ASTTrainer, default_ast_args
    seen = []
    orig = ops.conv3x3

    def spy(x, w_packed, bias, cout, *, upsample=1, pad_mode="zeros", want_pool=False, x2=None, **kw):
        n = int(x.shape[0]) + (int(x2.shape[0]) if x2 is not None else 0)
        shp = (n, int(x.shape[1]), int(x.shape[2]), int(x.shape[3]), cout, upsample, pad_mode, want_pool)
        if shp not in seen:
            seen.append(shp)
        return orig(x, w_packed, bias, cout, upsample=upsample, pad_mode=pad_mode, want_pool=want_pool, x2=x2, **kw)

    ops.conv3x3 = spy
    try:
        tr = ASTTrainer(default_ast_args(batch_size=batch), device="cuda",
                        ast=models.AST(attention=True).load_live_init(), graph=False)
        c = torch.from_numpy(synth.image(905, (batch, 3, size, size))).cuda()
        s = torch.from_numpy(synth.image(925, (batch, 3, size, size))).cuda()
        tr.train_step(c, s, record=False)
        torch.cuda.synchronize()
    finally:
        ops.conv3x3 = orig
    return seen


def key(n, cin, h, w, cout, up, pad, pool, kind=""):
    return f"{n}x{cin}x{h}x{w}->{cout} up{up} {pad}{' pool' if pool else ''}{kind}"


def dgrad_shapes(mode):
    """The fused input-gradient launches (ast_conv3x3_dgrad_f32) of one training step of `mode`
    ("train" = config 3, "ast", "ae"): (n, cout, H, W, cin, up, has_mask, has_pre, has_post), captured
    by spying functional.conv_input_grad in a live step."""
    from arbitrarystyletransfer_amd import functional as Fn
    seen = []
    orig = Fn.conv_input_grad

    def spy(dy, weight, upsample=1, pad_mode="zeros", in_scale=None, mask=None, add_pre=None, add_post=None):
        n, cout, H, W = (int(v) for v in dy.shape)
        fused = upsample == 2 or mask is not None or add_pre is not None or add_post is not None
        if fused and ops.pack_plan(n, W, False) == (1, 0):
            shp = (n, cout, H, W, int(weight.shape[1]), int(upsample), mask is not None, add_pre is not None,
                   add_post is not None)
            if shp not in seen:
                seen.append(shp)
        return orig(dy, weight, upsample, pad_mode, in_scale, mask, add_pre, add_post)

    Fn.conv_input_grad = spy
    try:
        {"train": adain_train_shapes, "ast": ast_shapes, "ae": ae_shapes}[mode]()
    finally:
        Fn.conv_input_grad = orig
    return seen


def time_dgrad(cfg, dy, packed, dx, mask, ap, aq, shp):
    from arbitrarystyletransfer_amd._lib import ptr, stream_ptr
    n, cout, H, W, cin, up = shp[:6]

    def launch():
        return lib().ast_conv3x3_dgrad_f32(cfg, ptr(dy), ptr(packed), ptr(dx), ptr(mask), ptr(ap), ptr(aq), n, cout, H,
                                           W, cin, up, stream_ptr(dy.device))
    if launch() != 0:
        return None
    for _ in range(2):
        launch()
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        launch()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


def tune_dgrad(mode, table, ncfg):
    """TUNE_DGRAD=train|ast|ae: time every configuration of each fused input-gradient launch of that
    training step; keys carry functional.dgrad_kind's suffix."""
    from arbitrarystyletransfer_amd import functional as Fn
    dev = torch.device("cuda:0")
    report = []
    for shp in dgrad_shapes(mode):
        n, cout, H, W, cin, up, hm, hp, hq = shp
        if os.environ.get("TUNE_CIN3") and cout > 3:  # the input-gradient conv's input is dy (cout channels)
            continue
        h, w = H // up, W // up
        dy = torch.from_numpy(synth.image(7, (n, cout, H, W))).to(dev)
        wt = torch.from_numpy(synth.conv_weight(8, cout, cin, 3)).to(dev)
        packed = Fn._TF.get(wt)
        dx = torch.empty((n, cin, h, w), device=dev)
        side = lambda on, seed: torch.from_numpy(synth.image(seed, (n, cin, h, w))).to(dev) if on else None  # noqa: E731
        mask, ap, aq = side(hm, 9), side(hp, 10), side(hq, 11)
        res = {}
        for cfg in cfg_list(ncfg):
            t = time_dgrad(cfg, dy, packed, dx, mask, ap, aq, shp)
            if t is not None:
                res[cfg] = t
        if not res:
            continue
        best = min(res, key=res.get)
        k = key(n, cout, H, W, cin, 1, "zeros", False, Fn.dgrad_kind(up))
        table[k] = best
        flops = 2 * n * H * W * cout * cin * 9
        row = {"shape": k, "best": best, "ms": res[best], "tflops": flops / res[best] / 1e9,
               "all_ms": {str(c): round(t, 4) for c, t in res.items()}}
        report.append(row)
        print(json.dumps(row), flush=True)
    return report


def cfg_list(ncfg):
    """TUNE_CFGS=a,b,...: time only these configurations (the others keep losing on these shapes)."""
    v = os.environ.get("TUNE_CFGS")
    return [int(c) for c in v.split(",") if int(c) < ncfg] if v else list(range(ncfg))


def time_cfg(cfg, x, wp, b, cout, up, pad, pool):
    args = dict(upsample=up, pad_mode=pad, want_pre=False, want_act=not pool, want_pool=pool, cfg=cfg)
    try:
        ops.conv3x3(x, wp, b, cout, **args)
    except Exception as e:
        if "unsupported" in str(e):
            return None
        raise
    for _ in range(2):
        ops.conv3x3(x, wp, b, cout, **args)
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        ops.conv3x3(x, wp, b, cout, **args)
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


def main():
    batch = int(os.environ.get("TUNE_BATCH", "8"))
    dev = torch.device("cuda:0")
    ncfg = lib().ast_conv3x3_num_configs()
    table = {}
    path = os.path.join(ROOT, "arbitrarystyletransfer_amd", "conv_tuning.json")
    if os.path.exists(path):
        table = json.load(open(path))
    report = []
    if os.environ.get("TUNE_DGRAD"):
        report = tune_dgrad(os.environ["TUNE_DGRAD"], table, ncfg)
        todo = []
    else:
        todo = ae_shapes() if os.environ.get("TUNE_AE") else adain_train_shapes() if os.environ.get("TUNE_TRAIN") \
            else ast_shapes() if os.environ.get("TUNE_AST") else shapes(batch)
        if os.environ.get("TUNE_NEW"):  # only shapes the table does not hold yet
            todo = [t for t in todo if key(*t) not in table]
        if os.environ.get("TUNE_SMALL"):  # only the shapes the direct VALU kernels serve (cin or cout <= 4)
            todo = [t for t in todo if t[1] <= 4 or t[4] <= 4]
        if os.environ.get("TUNE_CIN3"):  # only the shapes of the cin <= 3 kernels (configurations 42, 43)
            todo = [t for t in todo if t[1] <= 3]
    for shp in todo:
        n, cin, h, w, cout, up, pad, pool = shp
        x = torch.from_numpy(synth.image(5, (n, cin, h, w))).to(dev)
        wt = torch.from_numpy(synth.conv_weight(6, cout, cin, 3)).to(dev)
        wp = ops.pack_conv3x3(wt)
        b = torch.zeros(cout, device=dev)
        flops = 2 * n * h * up * w * up * cout * cin * 9
        res = {}
        for cfg in cfg_list(ncfg):
            t = time_cfg(cfg, x, wp, b, cout, up, pad, pool)
            if t is not None:
                res[cfg] = t
        best = min(res, key=res.get)
        k = key(*shp)
        table[k] = best
        row = {"shape": k, "best": best, "ms": res[best], "tflops": flops / res[best] / 1e9,
               "all_ms": {str(c): round(t, 4) for c, t in res.items()}}
        report.append(row)
        print(json.dumps(row), flush=True)
        del x, wt, wp
    with open(path, "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)
    extra = os.environ.get("TUNE_COPY")  # gpurun only returns gpurun_out/: keep a copy there
    if extra:
        with open(extra, "w") as f:
            json.dump(table, f, indent=1, sort_keys=True)
    tot = sum(r["ms"] for r in report)
    print(json.dumps({"total_ms_best": tot}))


if __name__ == "__main__":
    main()
