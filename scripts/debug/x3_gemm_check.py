"""mbtrain.gemm (split-bf16 path) on the AST step's shapes: repeatability (bitwise over 5 runs) and
error vs an fp64 torch matmul."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from arbitrarystyletransfer_amd import mbtrain as M  # noqa: E402

torch.manual_seed(0)
d = "cuda"
# (n, cin, cout, hw) pw convs of the AST step (batch 1..3 as in the DP test, and 8)
cases = [(1, 16, 96, 64 * 64), (2, 16, 96, 64 * 64), (3, 24, 144, 32 * 32), (1, 40, 240, 16 * 16), (3, 320, 80, 4 * 4),
         (1, 96, 16, 64 * 64), (2, 160, 40, 8 * 8), (8, 40, 160, 40 * 40), (1, 384, 128, 20 * 20), (3, 80, 320, 2 * 2)]
for (n, cin, cout, P) in cases:
    x = torch.randn(n, cin, P, device=d)
    w = torch.randn(cout, cin, device=d)
    g = torch.randn(n, cout, P, device=d)
    outs = []
    for rep in range(5):
        y = torch.empty(n, cout, P, device=d)
        M.gemm(w, x, y, cout, n * P, cin, 1, (0, cin, 1), (cin * P, P, 1), (cout * P, P, 1), fold_n=P)
        dx = torch.empty(n, cin, P, device=d)
        M.gemm(w, g, dx, cin, n * P, cout, 1, (0, 1, cin), (cout * P, P, 1), (cin * P, P, 1), fold_n=P)
        dw = torch.empty(cout, cin, device=d)
        M.gemm(g, x, dw, cout, cin, n * P, 1, (cout * P, P, 1), (cin * P, 1, P), (0, cin, 1),
               ksplit=M._ksplit(cout, cin, n * P), fold_k=P)
        torch.cuda.synchronize()
        outs.append((y.clone(), dx.clone(), dw.clone()))
    rep_ok = all(all(torch.equal(a, b) for a, b in zip(outs[0], o)) for o in outs[1:])
    yr = torch.einsum("mk,nkp->nmp", w.double(), x.double())
    dxr = torch.einsum("mk,nmp->nkp", w.double(), g.double())
    dwr = torch.einsum("nmp,nkp->mk", g.double(), x.double())
    err = [((a.double() - r).abs().max() / r.abs().max()).item() for a, r in zip(outs[0], (yr, dxr, dwr))]
    print((n, cin, cout, P), "repeatable" if rep_ok else "NOT REPEATABLE", " ".join(f"{e:.1e}" for e in err), flush=True)
