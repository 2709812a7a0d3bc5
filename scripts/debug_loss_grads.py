#!/usr/bin/env python3
"""Debug: d(loss component)/d(image) through the loss network, HIP vs CPU oracle autograd."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from arbitrarystyletransfer_amd import losses as L  # noqa: E402
from arbitrarystyletransfer_amd import models, synth  # noqa: E402
from oracle import ref_cpu as R  # noqa: E402

d = torch.device("cuda:0")
x = torch.from_numpy(synth.image(5, (2, 3, 64, 64)))
c = torch.from_numpy(synth.image(6, (2, 3, 64, 64)))
enc = [(torch.from_numpy(w), torch.from_numpy(b)) for w, b in synth.vgg_encoder_weights(1)]
lossnet = models.PretrainedEncoder().to(d).eval().requires_grad_(False)
names = R.LOSSNET_LAYERS


def cmp(tag, f_cpu, f_gpu):
    xr = x.clone().requires_grad_()
    f_cpu(xr).backward()
    xg = x.to(d).requires_grad_()
    f_gpu(xg).backward()
    a, b = xg.grad.cpu().double(), xr.grad.double()
    print(f"{tag:28s} rel_inf={float((a - b).abs().max() / b.abs().max()):.2e}  signflip={float(((a * b) < 0).double().mean()):.4f}")


cm_cpu = [m.detach() for m in R.vgg_encoder(c, enc, names)]
with torch.no_grad():
    cm_gpu = lossnet(c.to(d))
for i in range(6):
    cmp(f"content mvn layer {names[i]}", lambda t: R.compute_content_loss(R.mean_variance_norm(R.vgg_encoder(t, enc, names)[i]), R.mean_variance_norm(cm_cpu[i])),
        lambda t: L.content_mvn_loss(lossnet(t)[i], cm_gpu[i]))
    cmp(f"style layer {names[i]}", lambda t: R.compute_style_loss(R.vgg_encoder(t, enc, names)[i], cm_cpu[i]),
        lambda t: L.style_loss_weighted(lossnet(t)[i], cm_gpu[i]))
    cmp(f"sum layer {names[i]}", lambda t: R.vgg_encoder(t, enc, names)[i].sum() * 1e-3,
        lambda t: lossnet(t)[i].sum() * 1e-3)
cmp("all content, one call", lambda t: sum(R.compute_content_loss(R.mean_variance_norm(m), R.mean_variance_norm(r)) for m, r in zip(R.vgg_encoder(t, enc, names), cm_cpu)),
    lambda t: torch.stack([L.content_mvn_loss(m, r) for m, r in zip(lossnet(t), cm_gpu)]).sum())
cmp("all style, one call", lambda t: sum(R.compute_style_loss(m, r) for m, r in zip(R.vgg_encoder(t, enc, names), cm_cpu)),
    lambda t: torch.stack([L.style_loss_weighted(m, r) for m, r in zip(lossnet(t), cm_gpu)]).sum())


def both_cpu(t):
    ms = R.vgg_encoder(t, enc, names)
    return sum(R.compute_content_loss(R.mean_variance_norm(m), R.mean_variance_norm(r)) + R.compute_style_loss(m, r)
               for m, r in zip(ms, cm_cpu))


def both_gpu(t):
    ms = lossnet(t)
    return torch.stack([L.content_mvn_loss(m, r) + L.style_loss_weighted(m, r) for m, r in zip(ms, cm_gpu)]).sum()


cmp("content+style, one call", both_cpu, both_gpu)
for i in range(6):
    cmp(f"content+style {names[i]} only", lambda t: (lambda m: R.compute_content_loss(R.mean_variance_norm(m), R.mean_variance_norm(cm_cpu[i])) + R.compute_style_loss(m, cm_cpu[i]))(R.vgg_encoder(t, enc, names)[i]),
        lambda t: (lambda m: L.content_mvn_loss(m, cm_gpu[i]) + L.style_loss_weighted(m, cm_gpu[i]))(lossnet(t)[i]))
cmp("pixel content", lambda t: R.compute_content_loss(R.mean_variance_norm(t), R.mean_variance_norm(c)),
    lambda t: L.content_mvn_loss(t, c.to(d)))
cmp("pixel style", lambda t: R.compute_style_loss(t, c), lambda t: L.style_loss_weighted(t, c.to(d)))
cmp("tv", lambda t: R.tv_loss(t), lambda t: L.tv_loss(t))
