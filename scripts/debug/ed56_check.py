"""v6 (producer/consumer) vs v5 k5 expand+depthwise: the same block outputs bit for bit (the env
switch AST_MB_ED5 is read once per process, so each version runs in its own child).
python scripts/debug/ed56_check.py"""
import os
import subprocess
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CASES = [(40, 40, 4, (2, 70, 60)), (40, 24, 6, (1, 33, 100)), (24, 24, 6, (1, 5, 8)), (16, 16, 4, (2, 32, 28)),
         (40, 24, 6, (4, 256, 256))]

CHILD = r'''
import sys, torch
sys.path.insert(0, sys.argv[1])
from arbitrarystyletransfer_amd import synth
from arbitrarystyletransfer_amd.mobilenetv2 import DepthWiseConv
outs = []
for inp, oup, t, (n, h, w) in %r:
    blk = synth.live_init_(DepthWiseConv(inp, oup, 1, t, kernel_size=5, use_norm=True), 77 + inp)
    blk = blk.eval().cuda().to(torch.bfloat16)
    x = torch.from_numpy(synth.image(78 + inp, (n, inp, h, w)) * 2 - 0.7).cuda().to(torch.bfloat16)
    with torch.no_grad():
        outs.append(blk.run(x, None, 1).cpu())
torch.save(outs, sys.argv[2])
''' % (CASES,)


def run(ver, path):
    env = dict(os.environ, AST_MB_ED5=str(ver))
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, path], env=env, capture_output=True, text=True, timeout=300)
    if r.returncode:
        sys.exit(r.stdout[-2000:] + r.stderr[-2000:])
    return torch.load(path, weights_only=True)


with tempfile.TemporaryDirectory() as d:
    a, b = run(1, os.path.join(d, "v5.pt")), run(2, os.path.join(d, "v6.pt"))
    for c, x, y in zip(CASES, a, b):
        print(c, "equal" if torch.equal(x, y) else f"DIFFER max {float((x.float() - y.float()).abs().max()):.3e}")
