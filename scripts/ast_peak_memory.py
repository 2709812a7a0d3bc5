"""Peak device memory and time of AdaAttN's backward (models.py:81-115) in its materialised form (P
and dS as [n][Nq][Nk]) and in the flash form (csrc/adaattn_flash.hip): (1) the AdaAttN layer alone,
forward + backward at n = 8, C = 128 (the AST's channels) on 32^2, 64^2 and 128^2 maps, peak memory
of the backward; (2) one whole ASTTrainer step (train.py:186-300) at image sizes whose AdaAttN maps
are 64^2 and 128^2 (enc_out_layers at 1/8 of the image), whose peak is set by the train-mode encoder
and loss-network activations, not by the attention.
python scripts/ast_peak_memory.py [batch] [size ...]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys, time, torch
sys.path.insert(0, {root!r})
from arbitrarystyletransfer_amd import models, synth
from arbitrarystyletransfer_amd.train import ASTTrainer, default_ast_args
B, S = {b}, {s}
dev = torch.device("cuda")
tr = ASTTrainer(default_ast_args(batch_size=B), device=dev, ast=models.AST(attention=True).load_live_init(), graph=False)
c = torch.from_numpy(synth.image(905, (B, 3, S, S))).to(dev)
s = torch.from_numpy(synth.image(925, (B, 3, S, S))).to(dev)
tr.train_step(c, s)
torch.cuda.synchronize()
torch.cuda.reset_peak_memory_stats()
t0 = time.perf_counter()
for _ in range(3):
    out = tr.train_step(c, s)
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / 3 * 1e3
print(json.dumps({{"batch": B, "size": S, "map": S // 8, "peak_gb": torch.cuda.max_memory_allocated() / 2**30,
                  "ms_per_step": ms, "grad_norm": float(out["grad_norm"])}}))
"""


LAYER = r"""
import json, sys, time, torch
sys.path.insert(0, {root!r})
from arbitrarystyletransfer_amd import models, synth
n, C, H = 8, 128, {h}
dev = torch.device("cuda")
m = synth.live_init_(models.AdaAttN(C), 7).to(dev)
with torch.no_grad():
    m.W_q.weight.mul_(0.125)
    m.W_k.weight.mul_(0.125)
torch.manual_seed(0)
c = torch.rand(n, C, H, H, device=dev).requires_grad_()
s = torch.rand(n, C, H, H, device=dev).requires_grad_()
g = torch.rand(n, C, H, H, device=dev) - 0.5
(m(c, s) * g).sum().backward()
torch.cuda.synchronize()
out = m(c, s)
base = torch.cuda.memory_allocated()
torch.cuda.reset_peak_memory_stats()
t0 = time.perf_counter()
(out * g).sum().backward()
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) * 1e3
print(json.dumps({{"layer": "AdaAttN fwd+bwd", "n": n, "C": C, "map": H,
                  "backward_extra_gb": (torch.cuda.max_memory_allocated() - base) / 2**30, "backward_ms": ms,
                  "dWq_sum": float(m.W_q.weight.grad.sum())}}))
"""


def run(code, mode):
    env = dict(os.environ, AST_ADAATTN_FLASH=mode)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=280)
    if r.returncode != 0:
        print(r.stdout[-2000:], r.stderr[-3000:])
        sys.exit(1)
    d = json.loads(r.stdout.strip().splitlines()[-1])
    d["adaattn_backward"] = "flash" if mode == "1" else "materialised"
    print(json.dumps(d), flush=True)


def main():
    b = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    sizes = [int(x) for x in sys.argv[2:]] or [512, 1024]
    for h in (32, 64, 128):
        for mode in ("0", "1"):
            run(LAYER.format(root=ROOT, h=h), mode)
    for s in sizes:
        for mode in ("0", "1"):
            run(CHILD.format(root=ROOT, b=b, s=s), mode)


if __name__ == "__main__":
    main()
