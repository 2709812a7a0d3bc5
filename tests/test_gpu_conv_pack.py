"""GPU: side-by-side packing of small planes in ops.conv3x3 (csrc/pack.hip). Packing G images per
row band with zero gaps must give bit-identical outputs to the unpacked launch (the same
products summed in the same order per output pixel), including the fused max-pool (gap 2 keeps
images on even columns), the pre-activation output and a second batch (x2)."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from arbitrarystyletransfer_amd import ops, synth

pytestmark = pytest.mark.gpu

CASES = [(16, 32, 20, 20, 48, False, 0), (16, 32, 20, 20, 48, True, 0), (5, 16, 10, 10, 64, False, 3),
         (7, 24, 10, 12, 32, True, 0), (9, 8, 40, 40, 16, False, 0), (3, 8, 6, 9, 8, False, 2)]


def _run(x, x2, wp, b, cout, pool, pack):
    old = os.environ.get("AST_CONV_PACK")
    os.environ["AST_CONV_PACK"] = "1" if pack else "0"
    try:
        return ops.conv3x3(x, wp, b, cout, want_pre=True, want_act=not pool, want_pool=pool, x2=x2)
    finally:
        if old is None:
            del os.environ["AST_CONV_PACK"]
        else:
            os.environ["AST_CONV_PACK"] = old


@pytest.mark.parametrize("n,cin,h,w,cout,pool,n2", CASES)
def test_packed_equals_unpacked(n, cin, h, w, cout, pool, n2):
    dev = torch.device("cuda:0")
    x = torch.from_numpy(synth.image(41, (n, cin, h, w))).to(dev) - 0.5
    x2 = (torch.from_numpy(synth.image(42, (n2, cin, h, w))).to(dev) - 0.5) if n2 else None
    wt = torch.from_numpy(synth.conv_weight(43, cout, cin, 3)).to(dev)
    b = torch.linspace(-0.1, 0.1, cout, device=dev)
    wp = ops.pack_conv3x3(wt)
    assert ops.pack_plan(n + n2, w, pool)[0] > 1 or (n + n2, w) == (3 + 2, 9)
    got = _run(x, x2, wp, b, cout, pool, True)
    ref = _run(x, x2, wp, b, cout, pool, False)
    for g, r in zip(got, ref):
        assert (g is None) == (r is None)
        if g is not None:
            assert g.shape == r.shape and torch.equal(g, r)
    xa = torch.cat([x, x2]) if x2 is not None else x
    pre = F.conv2d(xa.cpu().double(), wt.cpu().double(), b.cpu().double(), padding=1)
    np.testing.assert_allclose(got[0].cpu().double().numpy(), pre.numpy(), rtol=0,
                               atol=1e-5 * float(pre.abs().max()))
    if pool:
        np.testing.assert_allclose(got[2].cpu().double().numpy(), F.max_pool2d(F.relu(pre), 2).numpy(), rtol=0,
                                   atol=1e-5 * float(pre.abs().max()))
