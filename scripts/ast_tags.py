"""Per-launch-tag breakdown of one ASTTrainer step (bench.py --mode ast-train shapes, eager)."""
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbitrarystyletransfer_amd import models, ops, synth  # noqa: E402
from arbitrarystyletransfer_amd.train import ASTTrainer, default_ast_args  # noqa: E402

B, S, K = int(os.environ.get("B", 8)), int(os.environ.get("S", 160)), 3
tr = ASTTrainer(default_ast_args(batch_size=B), device="cuda", ast=models.AST(attention=True).load_live_init(),
                graph=False)
c = torch.from_numpy(synth.image(905, (B, 3, S, S))).cuda()
s = torch.from_numpy(synth.image(925, (B, 3, S, S))).cuda()
for _ in range(2):
    tr.train_step(c, s, record=False)
torch.cuda.synchronize()
timer = ops.LaunchTimer()
with timer:
    for _ in range(K):
        tr.train_step(c, s, record=False)
torch.cuda.synchronize()
agg = defaultdict(lambda: [0.0, 0.0, 0])
for tag, fl, ms in timer.results():
    a = agg[tag]
    a[0] += fl
    a[1] += ms
    a[2] += 1
print(f"timed launches: {sum(a[1] for a in agg.values()) / K:.2f} ms/step")
fam = defaultdict(float)
for tag, (fl, ms, n) in agg.items():
    fam[" ".join(tag.split()[:2]) if tag.startswith("mbgemm") else tag.split()[0]] += ms / K
print({k: round(v, 3) for k, v in sorted(fam.items(), key=lambda kv: -kv[1])})
for tag, (fl, ms, n) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:70]:
    tf = fl / (ms * 1e-3) / 1e12 if fl > 0 else float("nan")
    print(f"{ms / K:8.3f} ms/step {n // K:4d}x  {tf:7.1f} TF  {tag}")
