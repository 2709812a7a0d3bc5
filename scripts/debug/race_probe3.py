"""Layer-by-layer version of race_probe2.py for the VGG encoder pass over content + style (x2):
every conv3x3 launch's outputs are kept and compared with the first repeat; prints, per layer,
how many repeats differ, so the first varying launch is named (run under concurrent GPU load)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from arbitrarystyletransfer_amd import models, ops, synth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 12
dev = torch.device("cuda")


def rnd(seed, shape):
    return torch.from_numpy(synth.uniform(seed, int(np.prod(shape))).astype(np.float32).reshape(shape)).to(dev)


net = models.AdaINStyleTransfer().to(dev)
enc = net.encoder
c, s = rnd(16, (2, 3, 128, 96)), rnd(17, (2, 3, 128, 96))
norm = enc._vgg_layers[0]


def walk():
    res = []
    cur, cur2 = c, s
    for idx, conv, want_pre, want_act, want_pool, collect in enc._plan():
        first = idx == 1
        pre, act, pool = ops.conv3x3(cur, enc._packed.get(conv), conv.bias, conv.out_channels, pad_mode="zeros",
                                     in_mean=norm.mean.view(-1) if first else None,
                                     in_std=norm.std.view(-1) if first else None,
                                     want_pre=want_pre, want_act=want_act, want_pool=want_pool, x2=cur2)
        n, cin, h, w = cur.shape[0] + (cur2.shape[0] if cur2 is not None else 0), cur.shape[1], cur.shape[2], cur.shape[3]
        G, gap = ops.pack_plan(n, w, want_pool)
        tag = f"conv_{idx} {cin}->{conv.out_channels} {h}x{w} n{n} pool{want_pool} pack G{G}"
        res.append((tag, [t.clone() for t in (pre, act, pool) if t is not None]))
        cur, cur2 = (pool if want_pool else act), None
    return res


with torch.no_grad():
    ref = walk()
    bad = [0] * len(ref)
    for _ in range(N):
        got = walk()
        for i, ((_, a), (_, b)) in enumerate(zip(got, ref)):
            if any(not torch.equal(x, y) for x, y in zip(a, b)):
                bad[i] += 1
    torch.cuda.synchronize()
for (tag, _), v in zip(ref, bad):
    print(f"{'VARIES' if v else 'same  '} {v:3d}/{N}  {tag}", flush=True)
