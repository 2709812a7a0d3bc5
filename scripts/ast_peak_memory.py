"""Peak device memory and time of one ASTTrainer step (train.py:186-300) with AdaAttN's backward in
its materialised form (P and dS as [n][Nq][Nk]) and in the flash form (csrc/adaattn_flash.hip), at
image sizes whose AdaAttN maps are 64^2 and 128^2 (enc_out_layers at 1/8 of the image).
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


def main():
    b = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    sizes = [int(x) for x in sys.argv[2:]] or [512, 1024]
    for s in sizes:
        for mode in ("0", "1"):
            env = dict(os.environ, AST_ADAATTN_FLASH=mode)
            r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, b=b, s=s)], env=env,
                               capture_output=True, text=True, timeout=280)
            if r.returncode != 0:
                print(r.stdout[-2000:], r.stderr[-3000:])
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            d["adaattn_backward"] = "flash" if mode == "1" else "materialised"
            print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
