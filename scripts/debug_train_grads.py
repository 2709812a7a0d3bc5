#!/usr/bin/env python3
"""Debug: compare the HIP training step with CPU autograd of the oracle on the golden step
inputs: gradient wrt the stylised image, and decoder parameter gradients (full loss and a plain
sum-of-squares loss through the decoder only)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from arbitrarystyletransfer_amd import models, synth  # noqa: E402
from arbitrarystyletransfer_amd.train import AdaINTrainer, default_args  # noqa: E402
from oracle import ref_cpu as R  # noqa: E402


def rel(a, b):
    a, b = a.detach().cpu().double(), b.detach().cpu().double()
    return float((a - b).abs().max() / b.abs().max())


g = np.load(os.path.join(ROOT, "tests/golden/train_step_64.npz"))
content, style = torch.from_numpy(g["content"]), torch.from_numpy(g["style"])
enc = [(torch.from_numpy(w), torch.from_numpy(b)) for w, b in synth.vgg_encoder_weights(1)]
dec = [(torch.from_numpy(w).clone().requires_grad_(), torch.from_numpy(b).clone().requires_grad_())
       for w, b in synth.vgg_decoder_weights(2)]
d = torch.device("cuda:0")

# (1) decoder only, loss = sum(y^2)/1000
with torch.no_grad():
    t = R.adain(R.vgg_encoder(content, enc[:9])[0], R.vgg_encoder(style, enc[:9])[0])
y = R.vgg_decoder(t, dec)
(y * y).sum().div(1000).backward()
ref = [p.grad.clone() for wb in dec for p in wb]
decg = models.VGGDecoder().to(d)
yg = decg(t.to(d))
(yg * yg).sum().div(1000).backward()
for i, (p, r) in enumerate(zip(decg.parameters(), ref)):
    print(f"decoder-only param{i}: rel_inf={rel(p.grad, r):.2e}")
print("decoder-only y rel", rel(yg, y))

# (2) full step: gradient wrt stylised
for wb in dec:
    for p in wb:
        p.grad = None
out = R.train_losses(content, style, enc, dec)
out["stylized"].retain_grad()
out["loss"].backward()
tr = AdaINTrainer(default_args(batch_size=2), device=d)
o = tr.compute_losses(content.to(d), style.to(d))
o["stylized"].retain_grad()
o["loss"].backward()
print("full: d loss/d stylized rel_inf", rel(o["stylized"].grad, out["stylized"].grad))
for i, (p, wb) in enumerate(zip(tr.params, [q for wb in dec for q in wb])):
    print(f"full param{i}: rel_inf={rel(p.grad, wb.grad):.2e}")
for k in ("content_loss", "style_loss", "lf_loss", "tv_loss", "loss"):
    print(k, float(o[k]), float(out[k]))

# (3) CPU loss gradient evaluated AT the GPU's stylised image (separates conditioning from bugs)
xs = o["stylized"].detach().cpu().clone().requires_grad_()
names = R.LOSSNET_LAYERS
cm = [m.detach() for m in R.vgg_encoder(content, enc, names)]
sm = [m.detach() for m in R.vgg_encoder(style, enc, names)]
tcs = R.vgg_encoder(xs, enc, names)
cl = sum(R.compute_content_loss(R.mean_variance_norm(a), R.mean_variance_norm(b)) for a, b in zip(tcs, cm))
cl = cl + R.compute_content_loss(R.mean_variance_norm(xs), R.mean_variance_norm(content)) * 0.1
sl = sum(R.compute_style_loss(a, b) * w for a, b, w in zip(tcs, sm, R.STYLE_WEIGHTS)) + R.compute_style_loss(xs, style)
(1.25 * cl + 0.5 * sl + 0.0006 * R.tv_loss(xs)).backward()
print("CPU grad at GPU stylised vs GPU grad: rel_inf", rel(o["stylized"].grad, xs.grad))
print("CPU grad at GPU stylised vs CPU grad at CPU stylised: rel_inf", rel(xs.grad, out["stylized"].grad))
