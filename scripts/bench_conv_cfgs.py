#!/usr/bin/env python3
"""Time conv3x3 configurations on the config-2 layer shapes (HIP events, median of 5 after 2
warm-ups) and check each against the default configuration's output.
python scripts/bench_conv_cfgs.py [cfg ...]   (default: 7 24 25 and the tuned/auto choice)"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
from arbitrarystyletransfer_amd import ops, synth  # noqa: E402
from tune_conv import shapes  # noqa: E402


def timed(fn):
    for _ in range(2):
        fn()
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


def main():
    cfgs = [int(c) for c in sys.argv[1:]] or [7, 24, 25]
    dev = torch.device("cuda")
    tot = {c: 0.0 for c in cfgs + [-1]}
    for (n, cin, h, w, cout, up, pad, pool) in shapes(8):
        if cin < 16:
            continue
        x = torch.from_numpy(synth.image(5, (n, cin, h, w))).to(dev)
        wp = ops.pack_conv3x3(torch.from_numpy(synth.conv_weight(6, cout, cin, 3)).to(dev))
        b = torch.from_numpy(synth.conv_bias(7, cout)).to(dev)
        flops = 2 * n * h * up * w * up * cout * cin * 9
        ref = ops.conv3x3(x, wp, b, cout, upsample=up, pad_mode=pad, want_pre=True, want_act=False, cfg=7)[0]
        row = f"{n}x{cin}x{h}x{w}->{cout} up{up} {pad}{' pool' if pool else ''}:"
        for c in cfgs + [-1]:
            f = lambda: ops.conv3x3(x, wp, b, cout, upsample=up, pad_mode=pad, want_pre=not pool, want_act=False,  # noqa
                                    want_pool=pool, cfg=c)
            try:
                ms = timed(f)
            except Exception as e:  # noqa
                row += f"  c{c} n/a"
                continue
            tot[c] += ms
            got = ops.conv3x3(x, wp, b, cout, upsample=up, pad_mode=pad, want_pre=True, want_act=False, cfg=c)[0]
            err = float((got - ref).abs().max() / ref.abs().max())
            row += f"  c{c} {ms:.3f}ms {flops / ms / 1e9:.0f}TF err{err:.1e}"
        print(row, flush=True)
    print("total ms per step:", {k: round(v, 3) for k, v in tot.items()})


if __name__ == "__main__":
    main()
