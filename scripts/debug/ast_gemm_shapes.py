"""Per-shape breakdown of the eager ASTTrainer step's timed launches (mbgemm / conv3x3 / ...):
HIP events around every launch (ops.LaunchTimer), aggregated over 3 steps, printed per step."""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from arbitrarystyletransfer_amd import models, ops, synth  # noqa: E402
from arbitrarystyletransfer_amd.train import ASTTrainer, default_ast_args  # noqa: E402

B, S, K = int(os.environ.get("B", 8)), int(os.environ.get("S", 160)), 3
dev = torch.device("cuda:0")
tr = ASTTrainer(default_ast_args(batch_size=B), device=dev, ast=models.AST(attention=True).load_live_init(), graph=False)
c = torch.from_numpy(synth.image(905, (B, 3, S, S))).to(dev)
s = torch.from_numpy(synth.image(925, (B, 3, S, S))).to(dev)
tr.train_step(c, s, record=False)
torch.cuda.synchronize()
timer = ops.LaunchTimer()
with timer:
    for _ in range(K):
        tr.train_step(c, s, record=False)
torch.cuda.synchronize()
agg = collections.defaultdict(lambda: [0.0, 0.0, 0])
for tag, fl, ms in timer.results():
    a = agg[tag]
    a[0] += fl / K
    a[1] += ms / K
    a[2] += 1
tot = sum(v[1] for v in agg.values())
fam = collections.defaultdict(float)
for t, v in agg.items():
    fam[" ".join(t.split()[:2])] += v[1]
print(f"timed launches: {tot:.2f} ms/step")
for f, ms in sorted(fam.items(), key=lambda kv: -kv[1]):
    print(f"  {ms:8.3f} ms  {f}")
for t, (fl, ms, n) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:60]:
    print(f"{ms:8.3f} ms {n // K:4d}x {fl / (ms * 1e-3) / 1e12 if ms else 0:7.1f} TF  {t}")
