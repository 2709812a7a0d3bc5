"""Run one AutoEncoder / AST training step several times from identical state in one process and
report gradients that are not bitwise identical (run two copies at once to add contention)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from arbitrarystyletransfer_amd import models, synth  # noqa: E402
from arbitrarystyletransfer_amd.train import (ASTTrainer, AutoencoderTrainer, default_ae_args,  # noqa: E402
                                              default_ast_args)

which = sys.argv[1] if len(sys.argv) > 1 else "ae"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
d = torch.device("cuda:0")
c = torch.from_numpy(synth.image(3, (B, 3, 64, 64))).to(d)
s = torch.from_numpy(synth.image(4, (B, 3, 64, 64))).to(d)
runs = []
poison = os.environ.get("POISON")   # "nan" | "rand": fill the allocator's free blocks before each run
for r in range(reps):
    if poison:
        torch.cuda.synchronize()
        junk = torch.empty(int(6e8), device=d)   # 2.4 GB carved into later allocations
        junk.fill_(float("nan")) if poison == "nan" else junk.uniform_(-1e3 * (r + 1), 1e3 * (r + 1))
        del junk
        torch.cuda.synchronize()
    torch.manual_seed(0)
    snap = {}
    if which == "ae":
        tr = AutoencoderTrainer(default_ae_args(batch_size=B), device=d, model=models.AutoEncoder().load_live_init())
        mod = tr.model
        orig = tr.ae_optim.step

        def step(orig=orig, mod=mod):
            snap.update({n: p.grad.detach().clone() for n, p in mod.named_parameters()})
            orig()
        tr.ae_optim.step = step
        tr.train_step(c)
    elif which == "astdp":   # rank 0's computation of tests/ast_dp_worker.py, in one process
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                        "tests"))
        import ast_dp_worker as W
        cc, ss = W.inputs()
        tr = W.make_trainer(d, lambda ps: None)
        mod = tr.ast
        tr.grad_hook = lambda ps, mod=mod: snap.update({n: p.grad.detach().clone() for n, p in mod.named_parameters()})
        tr.train_step(cc[:B].to(d), ss[:B].to(d))
    else:
        ast = models.AST(attention=True).load_live_init()
        tr = ASTTrainer(default_ast_args(batch_size=B), device=d, ast=ast,
                        grad_hook=lambda ps: None)
        mod = tr.ast
        tr.grad_hook = lambda ps, mod=mod: snap.update({n: p.grad.detach().clone() for n, p in mod.named_parameters()})
        tr.train_step(c, s)
    torch.cuda.synchronize()
    runs.append({k: v.cpu().numpy() for k, v in snap.items()})
bad = {}
for r in runs[1:]:
    for k in runs[0]:
        if not np.array_equal(runs[0][k], r[k]):
            e = float(np.abs(runs[0][k] - r[k]).max() / max(np.abs(runs[0][k]).max(), 1e-30))
            bad[k] = max(bad.get(k, 0.0), e)
nonfinite = [k for k in runs[0] if not all(np.isfinite(rr[k]).all() for rr in runs)]
print(f"{which} B={B} poison={poison}: {len(runs[0])} grads, {len(bad)} differ across {reps} runs, "
      f"{len(nonfinite)} non-finite {nonfinite[:5]}", flush=True)
for k, e in sorted(bad.items(), key=lambda kv: -kv[1])[:15]:
    print(f"   {e:.2e}  {k}")
