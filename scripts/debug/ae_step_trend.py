"""Per-step wall time of the AutoEncoder trainer over 40 steps (sync per step) and the allocator's
state: finds step-to-step growth (host-side caches, allocator churn)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.getcwd())
from arbitrarystyletransfer_amd import models, synth  # noqa: E402
from arbitrarystyletransfer_amd.train import AutoencoderTrainer, default_ae_args  # noqa: E402

B, S = 16, 160
tr = AutoencoderTrainer(default_ae_args(batch_size=B), device="cuda", model=models.AutoEncoder().load_live_init())
x = torch.from_numpy(synth.image(901, (B, 3, S, S))).cuda()
ts = []
for i in range(40):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.train_step(x, record=False)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
print(os.getcwd(), "ms/step by 5s:", [round(sum(ts[i:i + 5]) / 5, 2) for i in range(0, 40, 5)],
      "alloc MB", round(torch.cuda.memory_allocated() / 2**20), "reserved MB", round(torch.cuda.memory_reserved() / 2**20),
      "hipMalloc calls", torch.cuda.memory_stats().get("num_alloc_retries"), flush=True)
# host time of one step without sync (launch-bound share)
t0 = time.perf_counter()
for _ in range(5):
    tr.train_step(x, record=False)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print("5 steps: host issue", round((t1 - t0) * 200, 2), "ms/step, total", round((t2 - t0) * 200, 2), "ms/step", flush=True)
