"""Box fingerprint of a few training kernels: fixed inputs, output hashes. Run on several boxes;
a hash that differs between boxes names a kernel whose result depends on the machine (the DP
AutoEncoder step differed between boxes)."""
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from arbitrarystyletransfer_amd import functional as Fn, models, ops, synth  # noqa: E402


def h(t):
    return hashlib.sha1(t.detach().float().contiguous().cpu().numpy().tobytes()).hexdigest()[:12]


def rnd(seed, shape, scale=1.0):
    return torch.from_numpy((synth.uniform(seed, int(np.prod(shape))) * scale - 0.5 * scale).astype(np.float32)
                            .reshape(shape)).cuda()


p = torch.cuda.get_device_properties(0)
print("device", p.name, p.multi_processor_count, getattr(p, "gcnArchName", ""))
# the AE decoder's final conv (16 -> 3, reflect pad) forward and backward at 160^2, B = 16
x = rnd(1, (16, 16, 160, 160)).requires_grad_()
w = rnd(2, (3, 16, 3, 3), 0.2).requires_grad_()
b = rnd(3, (3,), 0.1).requires_grad_()
y = Fn.DecoderConvFn.apply(x, w, b, ops.pack_conv3x3(w.detach()), 1, False)
g = rnd(4, tuple(y.shape))
y.backward(g)
print("decconv y", h(y), "dx", h(x.grad), "dw", h(w.grad), "db", h(b.grad))
# a whole AutoEncoder backward on fixed inputs (single process)
ae = models.AutoEncoder().load_live_init().cuda().train()
img = torch.from_numpy(synth.image(9, (2, 3, 64, 64))).cuda()
out = ae(img)
(out.float() * rnd(5, tuple(out.shape))).sum().backward()
names = [n for n, _ in ae.named_parameters()]
grads = dict((n, q.grad) for n, q in ae.named_parameters() if q.grad is not None)
print("ae out", h(out), "grads", hashlib.sha1(b"".join(grads[n].cpu().numpy().tobytes() for n in names if n in grads)).hexdigest()[:12])
for n in names[-6:]:
    if n in grads:
        print("  ", n, h(grads[n]))
