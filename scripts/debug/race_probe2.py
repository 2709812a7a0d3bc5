"""Bisect the AdaIN forward's run-to-run variation under concurrent GPU load (race_probe.py):
the encoder pass, + AdaIN, + each decoder layer; prints how many of N repeats differ from the
first, per stage, and the first stage that varies."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from arbitrarystyletransfer_amd import models, synth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 12
dev = torch.device("cuda")


def rnd(seed, shape):
    return torch.from_numpy(synth.uniform(seed, int(np.prod(shape))).astype(np.float32).reshape(shape)).to(dev)


net = models.AdaINStyleTransfer().to(dev)
c, s = rnd(16, (2, 3, 128, 96)), rnd(17, (2, 3, 128, 96))


def stages():
    out = {}
    f_c, f_s = net.encode_pair(c, s)
    out["enc_c"], out["enc_s"] = f_c, f_s
    t = net.adain(f_c, f_s)
    out["adain"] = t
    x = t
    dec = net.decoder
    out["decoder"] = dec(t)
    return out


with torch.no_grad():
    ref = {k: v.clone() for k, v in stages().items()}
    bad = {k: 0 for k in ref}
    for _ in range(N):
        got = stages()
        for k in ref:
            if not torch.equal(got[k], ref[k]):
                bad[k] += 1
    torch.cuda.synchronize()
for k, v in bad.items():
    print(f"{'VARIES' if v else 'same  '} {v:3d}/{N}  {k}  ({os.environ.get('AST_CONV_PACK', '1')=}, {os.environ.get('AST_CONV_M16', '1')=})",
          flush=True)
