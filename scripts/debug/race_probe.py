"""Run-to-run bit equality of single ops while another process loads the GPU (start a bench in the
background first): each op runs N times on fixed inputs; prints the ops whose output changes.
A kernel whose result depends on wave scheduling shows here (tests/test_gpu_determinism.py runs
on an idle GPU and missed one)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from arbitrarystyletransfer_amd import functional as Fn, models, ops, synth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 12
dev = torch.device("cuda")


def rnd(seed, shape, scale=1.0, shift=0.0):
    return torch.from_numpy((synth.uniform(seed, int(np.prod(shape))) * scale + shift).astype(np.float32)
                            .reshape(shape)).to(dev)


cases = {}
x64 = rnd(1, (2, 64, 128, 96), 1.0, -0.3)
for cin, cout, hw, pad, up, pool in [(64, 64, (128, 96), "zeros", 1, True), (64, 128, (64, 48), "zeros", 1, False),
                                     (256, 256, (32, 24), "zeros", 1, False), (512, 512, (16, 12), "zeros", 1, False),
                                     (512, 256, (16, 12), "reflect", 2, False), (128, 64, (32, 24), "reflect", 2, False),
                                     (64, 64, (64, 48), "reflect", 1, False)]:
    x = rnd(cin + cout, (2, cin) + hw, 1.0, -0.2)
    w = rnd(cin * 3 + cout, (cout, cin, 3, 3), 0.1, -0.05)
    b = rnd(7 + cout, (cout,), 0.1)
    wp = ops.pack_conv3x3(w)
    cases[f"conv {cin}->{cout} {hw} {pad} up{up} pool{pool}"] = (
        lambda x=x, wp=wp, b=b, cout=cout, pad=pad, up=up, pool=pool:
        ops.conv3x3(x, wp, b, cout, upsample=up, pad_mode=pad, want_pre=True, want_act=True, want_pool=pool))
img = rnd(3, (2, 3, 128, 96), 1.0, 0.0)
w1 = rnd(4, (64, 3, 3, 3), 0.2, -0.1)
wp1 = ops.pack_conv3x3(w1)
b1 = rnd(5, (64,), 0.1)
mean = torch.tensor([0.485, 0.456, 0.406], device=dev)
std = torch.tensor([0.229, 0.224, 0.225], device=dev)
cases["conv_1 cin4 norm"] = lambda: ops.conv3x3(img, wp1, b1, 64, in_mean=mean, in_std=std, want_pre=True)
w3 = rnd(6, (3, 64, 3, 3), 0.1, -0.05)
wp3 = ops.pack_conv3x3(w3)
b3 = rnd(7, (3,), 0.1)
cases["smallc 64->3 reflect"] = lambda: ops.conv3x3(x64, wp3, b3, 3, pad_mode="reflect", want_pre=True, want_act=False)
sf = rnd(8, (2, 512, 16, 12), 1.0, 0.1)
cf = rnd(9, (2, 512, 16, 12), 1.0, 0.2)
cases["adain"] = lambda: ops.adain(cf, sf)
cases["channel_stats"] = lambda: ops.channel_stats(cf)
net = models.AdaINStyleTransfer().to(dev)
c, s = rnd(16, (2, 3, 128, 96)), rnd(17, (2, 3, 128, 96))
cases["AdaIN forward e2e"] = lambda: net(c, s)


def flat(o):
    if isinstance(o, (list, tuple)):
        return [t for x in o for t in flat(x)]
    return [o] if isinstance(o, torch.Tensor) else []


with torch.no_grad():
    for name, fn in cases.items():
        ref = [t.clone() for t in flat(fn())]
        bad = 0
        for _ in range(N):
            got = flat(fn())
            if any(not torch.equal(a, b) for a, b in zip(got, ref)):
                bad += 1
        torch.cuda.synchronize()
        print(f"{'VARIES' if bad else 'same  '} {bad:3d}/{N}  {name}", flush=True)
