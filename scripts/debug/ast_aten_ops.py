"""Which aten ops (not HIP-library calls) one eager ASTTrainer step runs, with the Python call
sites of the frequent ones: the source of the elementwise add / copy / fill launches in the trace."""
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.getcwd())
from arbitrarystyletransfer_amd import models, synth  # noqa: E402
from arbitrarystyletransfer_amd.train import ASTTrainer, default_ast_args  # noqa: E402

B, S = 8, 160
tr = ASTTrainer(default_ast_args(batch_size=B), device="cuda", ast=models.AST(attention=True).load_live_init(),
                graph=False)
c = torch.from_numpy(synth.image(905, (B, 3, S, S))).cuda()
s = torch.from_numpy(synth.image(925, (B, 3, S, S))).cuda()
tr.train_step(c, s, record=False)
ops = collections.Counter()
sites = collections.defaultdict(collections.Counter)


class Log(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func.overloadpacket)
        if any(a.is_cuda for a in args if isinstance(a, torch.Tensor)) or name.endswith(("zeros", "fill_", "empty")):
            ops[name] += 1
            if name in ("aten.add", "aten.copy_", "aten.fill_", "aten.zero_", "aten.cat", "aten.clone", "aten.mul",
                        "aten.add_", "aten.sum", "aten.zeros_like"):
                st = [f for f in traceback.extract_stack()[:-2] if "arbitrarystyletransfer_amd" in f.filename
                      or "torch/autograd" in f.filename]
                site = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in st[-3:]) or "?"
                sites[name][site] += 1
        return func(*args, **(kwargs or {}))


with Log():
    tr.train_step(c, s, record=False)
torch.cuda.synchronize()
for k, v in ops.most_common(25):
    print(f"{v:5d} {k}")
for k in sites:
    print("==", k)
    for site, n in sites[k].most_common(8):
        print(f"   {n:4d} {site}")
