"""Run-to-run determinism (race detection / determinism): every op whose reduction
is split across workgroups is run twice on the same inputs and must give the same bits.

The reference's CPU path is deterministic; here no floating-point partial sum meets another
through an atomic (csrc/det.h): split-K / pixel-split / tile partials go to a workspace and are
summed in a fixed order, scalar losses use the ordered loss accumulator, the soft histogram sums
exact fixed-point integers. Ops covered: gram split-K, conv3x3 wgrad (every kernel family), the
MobileNet training GEMM (K-split and batch-shared C), depthwise wgrad, SE backward, the SE pool of
every expand+depthwise kernel family, each loss value and gradient, and whole steps (AdaIN
forward, AdaINTrainer, AutoencoderTrainer, ASTTrainer, the config-5 MobileNet forward).
"""
import numpy as np
import pytest
import torch

from arbitrarystyletransfer_amd import functional as Fn
from arbitrarystyletransfer_amd import losses as L
from arbitrarystyletransfer_amd import mbtrain, models, synth
from arbitrarystyletransfer_amd.mobilenetv2 import DepthWiseConv

pytestmark = pytest.mark.gpu


def _flat(out):
    if torch.is_tensor(out):
        return [out]
    if isinstance(out, dict):
        return [t for k in sorted(out) for t in _flat(out[k])]
    if isinstance(out, (list, tuple)):
        return [t for o in out for t in _flat(o)]
    return []


def twice(fn):
    """fn() twice; every tensor it returns must be bitwise equal (NaN patterns included)."""
    a = [t.detach().clone() for t in _flat(fn())]
    torch.cuda.synchronize()
    b = [t.detach().clone() for t in _flat(fn())]
    torch.cuda.synchronize()
    assert len(a) == len(b) and a
    for i, (x, y) in enumerate(zip(a, b)):
        assert x.shape == y.shape, i
        same = torch.equal(x, y) or (x.is_floating_point() and torch.equal(torch.nan_to_num(x, 7.0),
                                                                          torch.nan_to_num(y, 7.0)))
        assert same, (i, tuple(x.shape), float((x.float() - y.float()).abs().max()))
    return a


def rnd(seed, shape, dev, scale=1.0, shift=0.0):
    return torch.from_numpy(synth.image(seed, shape) * scale + shift).to(dev)


@pytest.mark.parametrize("shape", [(2, 64, 64, 64), (3, 128, 40, 24), (1, 512, 32, 32), (4, 96, 9, 11)])
def test_gram_split_k(shape, hip_device):
    f = rnd(1, shape, hip_device)
    twice(lambda: L.gram_matrix(f))


WGRAD_CASES = [
    # n, cin, h, w, cout, up, pad: wgrad3 aligned, upsample, general, smallco (cout 3 / 16)
    (2, 64, 32, 32, 64, 1, "reflect"),
    (2, 128, 16, 16, 64, 2, "reflect"),
    (2, 24, 13, 9, 40, 1, "zeros"),
    (2, 64, 24, 40, 3, 1, "reflect"),
    (2, 16, 20, 20, 16, 1, "reflect"),
    # cout <= 3 on the split-bf16 MFMA form (wgrad_co3.hip: W % 16 == 0): ragged 64-column q tiles,
    # upsample, zero padding (no border slot), few / many input channels
    (2, 64, 24, 48, 3, 1, "reflect"),
    (1, 40, 18, 32, 3, 2, "reflect"),
    (2, 64, 10, 16, 2, 1, "zeros"),
    (1, 16, 20, 160, 3, 1, "reflect"),
    (1, 130, 9, 32, 1, 1, "reflect"),
]


@pytest.mark.parametrize("case", WGRAD_CASES)
def test_conv_wgrad(case, hip_device):
    """Bitwise run to run, and equal to torch's CPU weight / bias gradient (rel_inf 1e-5)."""
    n, cin, h, w, cout, up, pad = case
    x = rnd(2, (n, cin, h, w), hip_device)
    dy = rnd(3, (n, cout, h * up, w * up), hip_device, 2.0, -1.0)
    dw, db = twice(lambda: Fn.conv_weight_grad(x, dy, cout, up, pad))
    xc = x.double().cpu()
    if up == 2:
        xc = torch.nn.functional.interpolate(xc, scale_factor=2, mode="nearest")
    xc = torch.nn.functional.pad(xc, (1, 1, 1, 1), mode="reflect" if pad == "reflect" else "constant")
    ref = torch.nn.grad.conv2d_weight(xc, (cout, cin, 3, 3), dy.double().cpu())
    for got, want in ((dw, ref), (db, dy.double().cpu().sum(dim=(0, 2, 3)))):
        err = float((got.double().cpu() - want).abs().max() / want.abs().max())
        assert err <= 1e-5, err


def test_mbt_gemm_ksplit_and_shared(hip_device):
    d = hip_device
    A = rnd(4, (96, 20000), d, 2.0, -1.0)
    B = rnd(5, (20000, 48), d, 2.0, -1.0)

    def ksplit():
        C = torch.empty((96, 48), device=d)
        mbtrain.gemm(A, B, C, 96, 48, 20000, 1, (0, 20000, 1), (0, 48, 1), (0, 48, 1), ksplit=37)
        return C
    twice(ksplit)
    Ab = rnd(6, (5, 64, 300), d, 2.0, -1.0)
    Bb = rnd(7, (5, 300, 64), d, 2.0, -1.0)

    def shared():   # C shared across the batch (sCb = 0), accumulating onto a start value
        C = torch.full((64, 64), 0.5, device=d)
        mbtrain.gemm(Ab, Bb, C, 64, 64, 300, 5, (64 * 300, 300, 1), (300 * 64, 64, 1), (0, 64, 1), ksplit=3,
                     accumulate=True)
        return C
    twice(shared)


_GEMM_CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, '.')
from arbitrarystyletransfer_amd import mbtrain
d = np.load(sys.argv[1])
T = lambda k: torch.from_numpy(d[k]).cuda()
out = {}
# weight gradient of a 1x1 conv: dY [n][cout][P] . X^T, the image folded into K (k-contiguous A and B)
g, x = T('g'), T('x')
n, cout, P = g.shape
cin = x.shape[1]
dw = torch.empty((cout, cin), device='cuda')
mbtrain.gemm(g, x, dw, cout, cin, n * P, 1, (cout * P, P, 1), (cin * P, 1, P), (0, cin, 1), ksplit=5, fold_k=P)
out['wgrad'] = dw.cpu().numpy()
# batched, k-contiguous A only
A, B = T('A'), T('B')
C = torch.empty((A.shape[0], A.shape[1], B.shape[2]), device='cuda')
mbtrain.gemm(A, B, C, A.shape[1], B.shape[2], A.shape[2], A.shape[0], (A.shape[1] * A.shape[2], A.shape[2], 1),
             (B.shape[1] * B.shape[2], B.shape[2], 1), (A.shape[1] * B.shape[2], B.shape[2], 1))
out['batched'] = C.cpu().numpy()
np.savez(sys.argv[2], **out)
"""


def test_mbt_gemm_float4_staging_bit_identical(hip_device, tmp_path):
    """The float4 k-run staging of the training GEMM (AST_MBGEMM_VEC, csrc/mbtrain.hip) fills the
    same LDS tiles as the scalar staging: bit-identical products, on a folded-K weight gradient
    (ragged cout/cin, K split) and a batched product, each run in a child per setting."""
    import os
    import subprocess
    import sys
    rng = np.random.default_rng(3)
    f = lambda *s: (rng.random(s, dtype=np.float32) * 2 - 1)  # noqa: E731
    src = tmp_path / "in.npz"
    np.savez(src, g=f(3, 40, 1600), x=f(3, 72, 1600), A=f(2, 96, 512), B=f(2, 512, 70))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = []
    for vec in ("1", "0"):
        dst = tmp_path / f"out{vec}.npz"
        subprocess.run([sys.executable, "-c", _GEMM_CHILD, str(src), str(dst)], cwd=root, check=True, timeout=240,
                       env=dict(os.environ, AST_MBGEMM_VEC=vec))
        res.append(np.load(dst))
    for k in ("wgrad", "batched"):
        assert np.array_equal(res[0][k], res[1][k]), k
    ref = np.einsum("ncp,nkp->ck", np.load(src)["g"].astype(np.float64), np.load(src)["x"].astype(np.float64))
    assert np.abs(res[0]["wgrad"] - ref).max() <= 1e-4 * np.abs(ref).max()


@pytest.mark.parametrize("k,s", [(3, 1), (5, 2)])
def test_dw_and_se_backward(k, s, hip_device):
    torch.manual_seed(0)
    blk = DepthWiseConv(24, 24, s, 4, kernel_size=k, use_norm=True).to(hip_device).train()
    synth.live_init_(blk, 9)
    x = rnd(8, (3, 24, 33, 40), hip_device)
    g = rnd(9, (3, 24, (33 - 1) // s + 1, (40 - 1) // s + 1), hip_device, 2.0, -1.0)

    def step():
        blk.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_()
        y = blk(xi)
        y.backward(g)
        return [y, xi.grad] + [p.grad for p in blk.parameters()]
    twice(step)


ED_CASES = [
    # cin, cout, stride, ratio, k, h, w, dtype, up, split: the v4 / v4-stride-2 / v3 / v1 / ratio-1 kernels
    (16, 24, 1, 6, 3, 64, 64, torch.bfloat16, 1, False),
    (40, 40, 1, 6, 5, 48, 56, torch.bfloat16, 1, False),
    (24, 40, 2, 6, 5, 64, 64, torch.bfloat16, 1, False),
    (128, 128, 1, 3, 3, 32, 32, torch.bfloat16, 1, False),
    (40, 40, 1, 1, 3, 24, 32, torch.bfloat16, 2, False),
    (256, 128, 1, 3, 3, 16, 16, torch.bfloat16, 1, True),
    (16, 24, 1, 6, 3, 20, 28, torch.float32, 1, False),
    (16, 24, 2, 6, 3, 20, 28, torch.float32, 1, False),
]


@pytest.mark.parametrize("case", ED_CASES)
def test_expand_dw_se_pool(case, hip_device):
    cin, cout, s, ratio, k, h, w, dt, up, split = case
    blk = DepthWiseConv(cin, cout, s, ratio, kernel_size=k, use_norm=False, use_identity=not split)
    synth.live_init_(blk, 11)
    blk = blk.to(hip_device).to(dt).eval()
    x = rnd(10, (3, cin // 2 if split else cin, h, w), hip_device).to(dt)
    x2 = rnd(11, (3, cin // 2, h, w), hip_device).to(dt) if split else None
    with torch.no_grad():
        twice(lambda: blk.run(x, x2, up))


def test_loss_values_and_grads(hip_device):
    d = hip_device
    x = rnd(12, (2, 64, 40, 48), d, 3.0, -1.0)
    y = rnd(13, (2, 64, 40, 48), d, 3.0, -1.0)
    img = rnd(14, (2, 3, 96, 80), d, 1.4, -0.2)
    sty = rnd(15, (2, 3, 96, 80), d)

    def losses():
        xi, ii = x.clone().requires_grad_(), img.clone().requires_grad_()
        vals = [L.content_mvn_loss(xi, y), L.style_loss_weighted(xi, y, 0.75), L.compute_content_loss(xi, y),
                L.tv_loss(ii), L.out_of_range_loss(ii), L.pixel_mse_loss(ii, sty),
                L.compute_hist_loss(ii, sty, 1e-5)]
        torch.stack(vals).sum().backward()
        return vals + [xi.grad, ii.grad, Fn.soft_histogram(ii.detach())]
    twice(losses)


def test_adain_forward_e2e(hip_device):
    net = models.AdaINStyleTransfer().to(hip_device)
    c, s = rnd(16, (2, 3, 128, 96), hip_device), rnd(17, (2, 3, 128, 96), hip_device)
    with torch.no_grad():
        twice(lambda: net(c, s))


def _trainer_step(make, step):
    """A fresh trainer from the same initial state for each run."""
    def run():
        torch.manual_seed(0)
        tr = make()
        out = step(tr)
        params = tr.params if hasattr(tr, "params") else list(tr.model.parameters())
        return [out["loss"], out["grad_norm"]] + [p.detach() for p in params]
    return run


def test_adain_trainer_step(hip_device):
    from arbitrarystyletransfer_amd.train import AdaINTrainer, default_args
    c, s = rnd(18, (2, 3, 64, 64), hip_device), rnd(19, (2, 3, 64, 64), hip_device)
    twice(_trainer_step(lambda: AdaINTrainer(default_args(batch_size=2, full_losses=True), device=hip_device),
                        lambda tr: tr.train_step(c, s)))


def test_autoencoder_trainer_step(hip_device):
    from arbitrarystyletransfer_amd.train import AutoencoderTrainer, default_ae_args
    c = rnd(20, (2, 3, 64, 64), hip_device)
    twice(_trainer_step(lambda: AutoencoderTrainer(default_ae_args(batch_size=2), device=hip_device,
                                                   model=models.AutoEncoder().load_live_init()),
                        lambda tr: tr.train_step(c, record=False)))


def test_ast_trainer_step(hip_device):
    from arbitrarystyletransfer_amd.train import ASTTrainer, default_ast_args
    c, s = rnd(21, (2, 3, 64, 64), hip_device), rnd(22, (2, 3, 64, 64), hip_device)

    def run():
        torch.manual_seed(0)
        tr = ASTTrainer(default_ast_args(batch_size=2), device=hip_device,
                        ast=models.AST(attention=True).load_live_init())
        out = tr.train_step(c, s)
        return [out["loss"], out["grad_norm"]] + [p.detach() for p in tr.params] + list(tr.ast.buffers())
    twice(run)


def test_mobilenet_config5_forward(hip_device):
    ast = models.AST(exporting=True).load_live_init().eval().to(hip_device).to(torch.bfloat16)
    c = rnd(23, (2, 3, 256, 256), hip_device).to(torch.bfloat16)
    s = rnd(24, (2, 3, 256, 256), hip_device).to(torch.bfloat16)
    with torch.no_grad():
        y = twice(lambda: ast(c, s))[0]
        y1 = ast(c[1:], s[1:])
    assert torch.equal(y[1:], y1)   # and batch independence
    assert np.isfinite(y.float().cpu().numpy()).all()
