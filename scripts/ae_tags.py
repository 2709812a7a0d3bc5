"""Per-launch-tag breakdown of one AutoEncoder training step (bench.py --mode ae-train shapes)."""
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbitrarystyletransfer_amd import models, ops, synth  # noqa: E402
from arbitrarystyletransfer_amd.train import AutoencoderTrainer, default_ae_args  # noqa: E402

B, S = int(os.environ.get("B", 16)), int(os.environ.get("S", 160))
tr = AutoencoderTrainer(default_ae_args(batch_size=B), device="cuda", model=models.AutoEncoder().load_live_init())
x = torch.from_numpy(synth.image(901, (B, 3, S, S))).cuda()
for _ in range(3):
    tr.train_step(x, record=False)
torch.cuda.synchronize()
timer = ops.LaunchTimer()
with timer:
    for _ in range(5):
        tr.train_step(x, record=False)
torch.cuda.synchronize()
agg = defaultdict(lambda: [0.0, 0.0, 0])
for tag, fl, ms in timer.results():
    a = agg[tag]
    a[0] += fl
    a[1] += ms
    a[2] += 1
tot = sum(a[1] for a in agg.values()) / 5
print(f"timed launches: {tot:.2f} ms/step")
fam = defaultdict(float)
for tag, (fl, ms, n) in agg.items():
    fam[" ".join(tag.split()[:2]) if tag.startswith("mbgemm") else tag.split()[0]] += ms / 5
print({k: round(v, 3) for k, v in sorted(fam.items(), key=lambda kv: -kv[1])})
for tag, (fl, ms, n) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:60]:
    tf = fl / (ms * 1e-3) / 1e12 if fl > 0 else float("nan")
    print(f"{ms / 5:8.3f} ms/step {n // 5:4d}x  {tf:7.1f} TF  {tag}")
