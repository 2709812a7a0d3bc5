"""GPU parity for the MobileNet-variant training path (SURVEY.md §8f "next" #4; mbtrain.py,
csrc/mbtrain.hip): every autograd Function against torch CPU autograd of the same op, a whole
DepthWiseConv block (BatchNorm in training mode) against the same nn layers on the CPU, and one
AutoEncoder training step (train_autoencoder.py:124-165) against the reference's own step
(tests/golden/ae_train_step_64.npz).

Bars (fp32): single ops rel_inf <= 1e-4 (depthwise input grad: atomics, 2e-4); block outputs and
gradients 5e-4; the training step: losses 1e-4 relative, reconstruction 1e-4, gradients 1e-3 (of max(max|g|, 1e-5 |g|_2)),
updated parameters / running statistics 1e-4.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from arbitrarystyletransfer_amd import mbtrain as M
from arbitrarystyletransfer_amd import models, synth
from arbitrarystyletransfer_amd.mobilenetv2 import DepthWiseConv

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ae_train_step_64.npz")


def rel_inf(a, b):
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


def pair(*shape, scale=1.0):
    t = torch.randn(*shape) * scale
    return t.clone().requires_grad_(), t.cuda().requires_grad_()


@pytest.mark.parametrize("split,shape,cout", [(False, (2, 24, 9, 13), 40), (True, (2, 24, 9, 13), 40),
                                              (False, (3, 96, 5, 5), 130), (True, (4, 40, 20, 20), 72),
                                              # wide M, long K, odd K, large planes
                                              (False, (2, 16, 40, 64), 144), (False, (1, 144, 33, 32), 24),
                                              (False, (2, 17, 8, 12), 33), (True, (2, 96, 16, 16), 260)])
def test_pw_conv(split, shape, cout):
    torch.manual_seed(0)
    xc, xg = pair(*shape)
    wc, wg = pair(cout, shape[1] + (8 if split else 0), 1, 1)
    if split:
        x2c, x2g = pair(shape[0], 8, *shape[2:])
        yc = F.conv2d(torch.cat((xc, x2c), 1), wc)
        yg = M.PwConvFn.apply(xg, x2g, wg)
    else:
        yc = F.conv2d(xc, wc)
        yg = M.PwConvFn.apply(xg, None, wg)
    g = torch.randn_like(yc)
    yc.backward(g)
    yg.backward(g.cuda())
    assert rel_inf(yg, yc) <= 1e-4
    assert rel_inf(xg.grad, xc.grad) <= 1e-4 and rel_inf(wg.grad, wc.grad) <= 1e-4
    if split:
        assert rel_inf(x2g.grad, x2c.grad) <= 1e-4


@pytest.mark.parametrize("k,s,hw", [(3, 1, (10, 14)), (5, 1, (9, 12)), (3, 2, (11, 16)), (5, 2, (12, 9)), (5, 1, (3, 4)),
                                    (3, 2, (2, 3)), (5, 2, (50, 47)), (3, 1, (48, 50)),
                                    # the LDS-tiled kernels' tile shapes (csrc/mbt_dw.hip dw_plan): full
                                    # 160^2 planes, partial tiles in both axes, multi-tile wgrad groups
                                    (5, 1, (160, 160)), (3, 1, (80, 83)), (5, 2, (81, 80)), (3, 2, (40, 40)),
                                    (5, 1, (20, 20)), (3, 1, (131, 67))])
def test_dw_conv(k, s, hw):
    torch.manual_seed(1)
    c = 12
    xc, xg = pair(2, c, *hw)
    wc, wg = pair(c, 1, k, k)
    p = (k - 1) // 2
    yc = F.conv2d(F.pad(xc, (p, p, p, p), mode="reflect"), wc, stride=s, groups=c)
    yg = M.DwConvFn.apply(xg, wg, k, s)
    g = torch.randn_like(yc)
    yc.backward(g)
    yg.backward(g.cuda())
    assert rel_inf(yg, yc) <= 1e-4
    assert rel_inf(xg.grad, xc.grad) <= 2e-4 and rel_inf(wg.grad, wc.grad) <= 1e-4


@pytest.mark.parametrize("shape,offset", [((3, 16, 7, 5), 0.0), ((2, 6, 70, 71), 5.0)])
def test_batchnorm_train(shape, offset):
    torch.manual_seed(2)
    bnc = torch.nn.BatchNorm2d(shape[1])
    bnc.weight.data.uniform_(0.5, 1.5)
    bnc.bias.data.uniform_(-0.2, 0.2)
    bng = torch.nn.BatchNorm2d(shape[1]).cuda()
    bng.load_state_dict(bnc.state_dict())
    xc, xg = pair(*shape, scale=2.0)
    xc.data += offset
    xg.data += offset
    yc = bnc(xc)
    yg = M.BatchNormTrainFn.apply(xg, bng.weight, bng.bias, bng)
    g = torch.randn_like(yc)
    yc.backward(g)
    yg.backward(g.cuda())
    assert rel_inf(yg, yc) <= 1e-4 and rel_inf(xg.grad, xc.grad) <= 1e-4
    assert rel_inf(bng.weight.grad, bnc.weight.grad) <= 1e-4 and rel_inf(bng.bias.grad, bnc.bias.grad) <= 1e-4
    assert rel_inf(bng.running_mean, bnc.running_mean) <= 1e-5 and rel_inf(bng.running_var, bnc.running_var) <= 1e-5
    assert int(bng.num_batches_tracked) == int(bnc.num_batches_tracked) == 1


@pytest.mark.parametrize("shape", [(3, 16, 7, 5), (2, 24, 40, 40)])
def test_batchnorm_hardswish_fused(shape):
    """BatchNormTrainFn(act=1): BN -> Hardswish in one apply pass, the Hardswish derivative taken
    inside the backward's passes. Against torch, and bit-identical to the unfused chain (same
    affine expression recomputed, same sums)."""
    torch.manual_seed(5)
    bnc = torch.nn.BatchNorm2d(shape[1])
    bnc.weight.data.uniform_(0.5, 1.5)
    bnc.bias.data.uniform_(-0.2, 0.2)
    bns = [torch.nn.BatchNorm2d(shape[1]).cuda() for _ in range(2)]
    for b in bns:
        b.load_state_dict(bnc.state_dict())
    xc, xg = pair(*shape, scale=3.0)
    yc = F.hardswish(bnc(xc))
    g = torch.randn_like(yc)
    yc.backward(g)
    xg2 = xg.detach().clone().requires_grad_()
    yf = M.BatchNormTrainFn.apply(xg, bns[0].weight, bns[0].bias, bns[0], 1)
    yu = M.HardswishFn.apply(M.BatchNormTrainFn.apply(xg2, bns[1].weight, bns[1].bias, bns[1], 0))
    yf.backward(g.cuda())
    yu.backward(g.cuda())
    assert rel_inf(yf, yc) <= 1e-4 and rel_inf(xg.grad, xc.grad) <= 1e-4
    assert rel_inf(bns[0].weight.grad, bnc.weight.grad) <= 1e-4 and rel_inf(bns[0].bias.grad, bnc.bias.grad) <= 1e-4
    assert torch.equal(yf, yu) and torch.equal(xg.grad, xg2.grad)
    assert torch.equal(bns[0].weight.grad, bns[1].weight.grad) and torch.equal(bns[0].bias.grad, bns[1].bias.grad)
    assert torch.equal(bns[0].running_var, bns[1].running_var)


@pytest.mark.parametrize("k,s,hw", [(5, 1, (40, 40)), (3, 2, (21, 18)), (3, 1, (160, 160))])
def test_hardswish_fused_into_dw_and_se(k, s, hw):
    """DwConvFn / SEFn with act=1 (the block's Hardswish applied while staging, its derivative in
    the gradient pass) are bit-identical to HardswishFn followed by the unfused op."""
    torch.manual_seed(6)
    c = 16
    x = (torch.randn(2, c, *hw) * 3).cuda()
    w = torch.randn(c, 1, k, k).cuda() * 0.3
    fc1w, fc1b = torch.randn(8, c).cuda() * 0.3, torch.randn(8).cuda() * 0.1
    fc2w, fc2b = torch.randn(c, 8).cuda() * 0.3, torch.randn(c).cuda() * 0.1 + 0.5
    res = []
    for fused in (True, False):
        xs = x.clone().requires_grad_()
        ws, p1, q1, p2, q2 = (t.clone().requires_grad_() for t in (w, fc1w, fc1b, fc2w, fc2b))
        if fused:
            d = M.DwConvFn.apply(xs, ws, k, s, 1)
            y = M.SEFn.apply(d, p1, q1, p2, q2, 1)
        else:
            d = M.DwConvFn.apply(M.HardswishFn.apply(xs), ws, k, s, 0)
            y = M.SEFn.apply(M.HardswishFn.apply(d), p1, q1, p2, q2, 0)
        g = torch.randn(y.shape, generator=torch.Generator().manual_seed(7)).cuda()
        y.backward(g)
        res.append((y.detach(), xs.grad, ws.grad, p1.grad, q1.grad, p2.grad, q2.grad))
    for a, b in zip(*res):
        assert torch.equal(a, b)
    # and against torch
    xc = x.cpu().requires_grad_()
    pp = (k - 1) // 2
    dc = F.conv2d(F.pad(F.hardswish(xc), (pp, pp, pp, pp), mode="reflect"), w.cpu(), stride=s, groups=c)
    a2 = F.hardswish(dc)
    gate = torch.clamp(F.linear(F.relu(F.linear(a2.mean((2, 3)), fc1w.cpu(), fc1b.cpu())), fc2w.cpu(), fc2b.cpu()), 0, 1)
    yc = a2 * gate[:, :, None, None]
    yc.backward(torch.randn(yc.shape, generator=torch.Generator().manual_seed(7)))
    assert rel_inf(res[0][0], yc) <= 1e-4 and rel_inf(res[0][1], xc.grad) <= 2e-4


def test_eltwise_and_se():
    torch.manual_seed(3)
    xc, xg = pair(2, 8, 6, 7, scale=3.0)
    yc = F.hardswish(xc)
    yg = M.HardswishFn.apply(xg)
    g = torch.randn_like(yc)
    yc.backward(g)
    yg.backward(g.cuda())
    assert rel_inf(yg, yc) <= 1e-6 and rel_inf(xg.grad, xc.grad) <= 1e-6
    xc, xg = pair(2, 5, 4, 3)
    yc = F.interpolate(xc, scale_factor=2, mode="nearest")
    yg = M.Upsample2Fn.apply(xg)
    g = torch.randn_like(yc)
    yc.backward(g)
    yg.backward(g.cuda())
    assert rel_inf(yg, yc) == 0 and rel_inf(xg.grad, xc.grad) <= 1e-6
    # SELayer (mobilenetv2.py:72-81)
    c, red = 24, 8
    xc, xg = pair(3, c, 5, 6)
    w1c, w1g = pair(red, c, scale=0.3)
    b1c, b1g = pair(red, scale=0.3)
    w2c, w2g = pair(c, red, scale=0.3)
    b2c, b2g = pair(c, scale=0.3)
    b2c.data += 0.5
    b2g.data += 0.5
    gate = F.hardtanh(F.linear(F.relu(F.linear(xc.mean(dim=(2, 3)), w1c, b1c)), w2c, b2c), 0.0, 1.0)
    yc = xc * gate[:, :, None, None]
    yg = M.SEFn.apply(xg, w1g, b1g, w2g, b2g)
    g = torch.randn_like(yc)
    yc.backward(g)
    yg.backward(g.cuda())
    assert rel_inf(yg, yc) <= 1e-5
    for a, b in ((xg, xc), (w1g, w1c), (b1g, b1c), (w2g, w2c), (b2g, b2c)):
        assert rel_inf(a.grad, b.grad) <= 1e-4


def _cpu_block(blk, x):
    """The same block's nn layers on the CPU (the reference forward, SELayer written out)."""
    h = x
    for layer in blk._layers:
        if layer.__class__.__name__ == "SELayer":
            y = h.mean(dim=(2, 3))
            y = layer.fc(y)
            h = h * y[:, :, None, None]
        else:
            h = layer(h)
    return h + x if blk.identity else h


@pytest.mark.parametrize("cfg", [(16, 16, 1, 6, 3, True, 12), (24, 40, 2, 6, 5, True, 16), (40, 40, 1, 1, 3, False, 10),
                                 (40, 24, 1, 4, 5, False, 11)])
def test_block_train(cfg):
    inp, oup, s, t, k, norm, hw = cfg
    blk = synth.live_init_(DepthWiseConv(inp, oup, s, t, kernel_size=k, use_norm=norm), 31).train()
    ref = synth.live_init_(DepthWiseConv(inp, oup, s, t, kernel_size=k, use_norm=norm), 31).train()
    blkg = blk.cuda()
    x = torch.rand(2, inp, hw, hw) * 2 - 0.5
    xc = x.clone().requires_grad_()
    xg = x.cuda().requires_grad_()
    yc = _cpu_block(ref, xc)
    yg = blkg(xg)
    g = torch.randn_like(yc)
    yc.backward(g)
    yg.backward(g.cuda())
    assert rel_inf(yg, yc) <= 5e-4
    assert rel_inf(xg.grad, xc.grad) <= 5e-4
    for (n1, p1), (n2, p2) in zip(blkg.named_parameters(), ref.named_parameters()):
        assert rel_inf(p1.grad, p2.grad) <= 5e-4, n1
    for (n1, b1), (n2, b2) in zip(blkg.named_buffers(), ref.named_buffers()):
        if "running" in n1:
            assert rel_inf(b1, b2) <= 1e-5, n1


def test_autoencoder_train_step_golden():
    from arbitrarystyletransfer_amd.train import AutoencoderTrainer, default_ae_args
    g = np.load(GOLDEN)
    ae = models.AutoEncoder().load_live_init()
    tr = AutoencoderTrainer(default_ae_args(batch_size=2), device="cuda", model=ae)
    snap, p0 = {}, {}
    orig_step = tr.ae_optim.step

    def step_with_snapshot():
        for n, p in tr.model.named_parameters():
            snap[n] = p.grad.detach().clone()
            p0[n] = p.detach().clone()
        orig_step()

    tr.ae_optim.step = step_with_snapshot
    content = torch.from_numpy(g["content"]).cuda()
    out = tr.train_step(content)
    for k in ("recon_loss", "content_loss", "loss"):
        np.testing.assert_allclose(out[k].item(), float(g[k]), rtol=1e-4, err_msg=k)
    assert rel_inf(out["recon"], g["recon"]) <= 1e-4
    norm = out["grad_norm"].item()
    np.testing.assert_allclose(norm, float(g["grad_norm"]), rtol=1e-3)
    coef = min(1.0, 10.0 / (norm + 1e-6))
    lr, eps = 2e-4, 1e-7

    def sub(t, ref):
        t = t.reshape(-1)
        return (t if t.numel() == ref.size else t[::17]).reshape(ref.shape)

    worst, far, total = 0.0, 0, 0
    rows = []
    for n, p in tr.model.named_parameters():
        ref = g[f"grad:{n}"]
        # a conv bias in front of a BatchNorm has an exactly-zero gradient; both sides hold rounding
        # noise (~1e-9) there, so errors are taken relative to max(max|g|, 1e-5 * total norm)
        e = float(np.abs(sub(snap[n], ref).cpu().numpy() - ref).max()) / max(float(np.abs(ref).max()), 1e-5 * norm)
        rows.append((e, float(np.abs(ref).max()), n))
        worst = max(worst, e)
        # Adam's first step is lr * g / (|g| + eps): our update from our own (clipped) gradient
        gc = snap[n] * coef
        want = p0[n] - lr * gc / (gc.abs() + eps)
        assert rel_inf(p.detach(), want) <= 1e-5, n
        # and the reference's parameters: the update is sign-like, so a gradient element within
        # rounding of zero may step the other way (|diff| <= 2 lr); elements whose reference
        # gradient is clearly non-zero (> 1e-3 of the tensor's max and > 1e-6) agree to 1e-6
        pref = g[f"param:{n}"]
        d = np.abs(sub(p.detach(), pref).cpu().numpy() - pref)
        assert d.max() <= 2.05 * lr, n
        sure = np.abs(ref) > max(1e-3 * float(np.abs(ref).max()), 1e-6)
        far += int((d[sure] > 1e-6).sum())
        total += int(sure.sum())
    assert worst <= 1e-3, (worst, worst_key)
    assert far <= 1e-4 * total, (far, total)
    for n, b in tr.model.named_buffers():
        if f"buf:{n}" in g.files:
            assert rel_inf(b, g[f"buf:{n}"]) <= 1e-4, n
    print(f"grad worst {worst:.2e} ({sorted(rows)[-1][2]}); params off by > 1e-6: {far}/{total}")


def test_autoencoder_dp_syncbn_step_golden(tmp_path):
    """Two ranks (torch.distributed.run, gloo on the one GPU), one image each, SyncBatchNorm and
    the averaged gradient arena: the step equals the reference's single-process step on both
    images (train_autoencoder.py)."""
    import socket
    import subprocess
    import sys
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "dp.npz")
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ae_dp_worker.py")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", f"--master-port={port}", worker, out],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    got = np.load(out)
    if os.environ.get("AST_TEST_DUMP"):   # debugging aid: keep the ranks' result for offline diffing
        import shutil
        shutil.copy(out, os.path.join(os.environ["AST_TEST_DUMP"], f"dp_{os.getpid()}_{port}.npz"))
    g = np.load(GOLDEN)
    for i, k in enumerate(("recon_loss", "content_loss", "loss")):
        np.testing.assert_allclose(got["losses"][i], float(g[k]), rtol=1e-4, err_msg=k)
    assert rel_inf(got["recon"], g["recon"]) <= 1e-4
    norm = float(got["grad_norm"])
    np.testing.assert_allclose(norm, float(g["grad_norm"]), rtol=1e-3)
    worst, worst_key = 0.0, None
    for key in g.files:
        if not key.startswith("grad:"):
            continue
        ref = g[key]
        mine = got[key].reshape(-1)
        mine = (mine if mine.size == ref.size else mine[::17]).reshape(ref.shape)
        e = float(np.abs(mine - ref).max()) / max(float(np.abs(ref).max()), 1e-5 * norm)
        if e > worst:
            worst, worst_key = e, key
        pref = g["param:" + key[5:]]
        pv = got["param:" + key[5:]].reshape(-1)
        pv = (pv if pv.size == pref.size else pv[::17]).reshape(pref.shape)
        assert np.abs(pv - pref).max() <= 2.05 * 2e-4, key
    assert worst <= 1e-3, (worst, worst_key)
    for key in g.files:
        if key.startswith("buf:"):
            assert rel_inf(got[key], g[key]) <= 1e-4, key


def test_autoencoder_trainer_loop_checkpoint(tmp_path):
    """AutoencoderTrainer.train / validate / save / load (train_autoencoder.py:88-120): the loop
    records the reference's train_dict keys, ae.pth holds {"AE", "optim"}, and a reloaded trainer
    continues identically (up to float-atomic summation order)."""
    from arbitrarystyletransfer_amd.train import AutoencoderTrainer, default_ae_args
    imgs = torch.from_numpy(synth.image(77, (4, 3, 32, 32)))

    def it():
        while True:
            yield imgs[:2]

    args = default_ae_args(batch_size=2, train_iter=3, save_dir=str(tmp_path))
    tr = AutoencoderTrainer(args, content_iter=it(), val_loader=it(), device="cuda",
                            model=models.AutoEncoder().load_live_init())
    tr.train()
    tr.validate()
    assert len(tr.train_dict["train_loss"]) == 3 and len(tr.train_dict["perp_loss"]) == 3
    assert len(tr.train_dict["val_loss"]) == 1 and np.isfinite(tr.train_dict["val_loss"][0])
    assert tr.model.training
    tr.save()
    saved = torch.load(os.path.join(str(tmp_path), "ae.pth"), weights_only=True)
    assert set(saved) == {"AE", "optim"}
    tr2 = AutoencoderTrainer(args, device="cuda", model=models.AutoEncoder())
    tr2.load()
    for (n1, p1), (n2, p2) in zip(tr.model.state_dict().items(), tr2.model.state_dict().items()):
        assert n1 == n2 and torch.equal(p1, p2), n1
    x = imgs[2:].cuda()
    o1 = tr.train_step(x, record=False)
    o2 = tr2.train_step(x, record=False)
    # float atomics in the loss and weight-gradient reductions: equal up to summation order
    np.testing.assert_allclose(o1["loss"].item(), o2["loss"].item(), rtol=1e-6)
    for p1, p2 in zip(tr.model.parameters(), tr2.model.parameters()):
        assert float((p1 - p2).detach().abs().max()) <= 2.05 * 2e-4   # Adam steps agree (sign-like first moments)
        assert rel_inf(p1, p2) <= 1e-3
