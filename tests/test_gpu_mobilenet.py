"""GPU parity of the MobileNet-style variant against the CPU oracle
(oracle/ref_cpu.py mb_*) and the golden vectors made by the reference's own modules.

Tolerances (rel_inf = max|a-b| / max|b|, each map against its own scale):
  fp32 single block 5e-5; fp32 encoder/decoder chains 1e-4 per map; fp32 end-to-end 1e-3 (north star).
  bf16 storage (fp32 arithmetic, config 5) against the fp32 oracle run on the same bf16-rounded
  weights and inputs: single block / AdaIN / ada_out / image conv 2e-2, encoder and decoder chains
  4e-2 per map (measured 0.3-1.3%, scripts/mb_bf16_errors.py); the end-to-end ada_out input is
  bounded at 0.2 only, because AdaIN divides by small content stds (see check_bf16_segments).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from arbitrarystyletransfer_amd import models, synth
from arbitrarystyletransfer_amd.mobilenetv2 import DepthWiseConv
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu

BLOCK_TOL = 5e-5
CHAIN_TOL = 1e-4
E2E_TOL = 1e-3
BF16_BLOCK_TOL = 2e-2
BF16_CHAIN_TOL = 4e-2
BF16_E2E_T_TOL = 0.2


def rel_inf(a, b):
    a = np.asarray(a.detach().float().cpu() if torch.is_tensor(a) else a, np.float64)
    b = np.asarray(b.detach().float().cpu() if torch.is_tensor(b) else b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


def cpu_sd(module):
    return {k: v.detach().float().cpu() for k, v in module.state_dict().items()}


BLOCKS = [
    # inp, oup, stride, expand, k, use_norm, use_identity, (n, h, w), up
    (16, 16, 1, 6, 3, True, True, (2, 20, 36), 1),
    (16, 24, 2, 6, 3, True, True, (1, 33, 40), 1),
    (24, 40, 2, 6, 5, True, True, (1, 32, 30), 1),
    (40, 40, 1, 4, 5, True, True, (2, 16, 24), 1),
    (96, 128, 1, 3, 3, True, True, (1, 8, 8), 1),
    (128, 128, 1, 3, 3, True, True, (1, 10, 6), 1),
    (80, 40, 1, 4, 3, False, True, (1, 16, 16), 1),
    (40, 24, 1, 6, 5, False, True, (1, 64, 64), 1),
    (40, 40, 1, 1, 3, False, True, (1, 9, 13), 2),     # DecoderBlock upsample + ratio-1 block
    (40, 40, 1, 1, 3, False, True, (2, 16, 24), 2),    # upsample, whole 8-pixel runs (vector pw epilogue)
    (24, 24, 1, 1, 3, False, True, (2, 12, 20), 1),    # ratio-1, no upsample
    (96, 80, 1, 4, 5, False, True, (1, 16, 16), 1),
    (16, 16, 1, 6, 3, False, True, (1, 3, 5), 1),      # tiny map (reflect pad on 3 rows)
    (20, 20, 1, 6, 3, False, True, (2, 12, 40), 1),    # hidden 120: a partial last 16-channel chunk
    (36, 36, 1, 3, 5, True, True, (1, 19, 70), 1),     # hidden 108, k5, ragged tiles both ways
    (20, 24, 2, 6, 3, False, True, (2, 70, 92), 1),    # stride 2: hidden 120, 4 strips, odd output height
    (24, 40, 2, 6, 5, True, True, (1, 66, 124), 1),    # k5 stride 2: 2 bands of output rows, 5 strips
    # k5 stride 1 with cin <= 48 and W % 4 == 0: the MFMA depthwise (v5, csrc/mb_ed5.hip)
    (40, 40, 1, 4, 5, False, True, (2, 70, 60), 1),    # 3 bands (last ragged), last strip 4 columns wide
    (40, 24, 1, 6, 5, True, True, (1, 33, 100), 1),    # hidden 240: a half-filled last 32-channel chunk
    (24, 24, 1, 6, 5, False, True, (1, 5, 8), 1),      # map smaller than one tile (reflect on 5 rows)
    (16, 16, 1, 4, 5, True, True, (2, 32, 28), 1),     # exactly one tile, one K-step
    (20, 16, 1, 3, 5, False, True, (1, 40, 44), 1),    # hidden 60 (past hid16 = 64 in the last chunk), 2 K-steps
]


def run_block(case, dev, dtype, seed):
    inp, oup, s, t, k, norm, ident, (n, h, w), up = case
    blk = synth.live_init_(DepthWiseConv(inp, oup, s, t, kernel_size=k, use_norm=norm, use_identity=ident), seed)
    blk = blk.eval().to(dev).to(dtype)
    x = torch.from_numpy(synth.image(seed + 1, (n, inp, h, w)) * 2 - 0.7)
    with torch.no_grad():
        y = blk.run(x.to(dev).to(dtype), None, up)
        xr = x.to(dtype).float()
        if up == 2:
            xr = F.interpolate(xr, scale_factor=2, mode="nearest")
        ref = R.mb_block(xr, cpu_sd(blk), "", inp, oup, s, t, k, norm, ident)
    return y, ref


@pytest.mark.parametrize("case", BLOCKS)
def test_block_fp32(case, hip_device):
    y, ref = run_block(case, hip_device, torch.float32, 900 + case[0] + case[1])
    torch.cuda.synchronize()
    assert y.dtype == torch.float32 and y.shape == ref.shape
    assert rel_inf(y, ref) <= BLOCK_TOL


@pytest.mark.parametrize("case", BLOCKS)
def test_block_bf16(case, hip_device):
    y, ref = run_block(case, hip_device, torch.bfloat16, 950 + case[0] + case[1])
    assert y.dtype == torch.bfloat16
    assert rel_inf(y, ref) <= BF16_BLOCK_TOL


FUSED_CASES = [
    # inp, oup, expand, use_norm, (n, h, w): the stride-1 k3 expand blocks of the fused pair
    (16, 16, 6, True, (2, 20, 36)),
    (16, 16, 6, False, (1, 70, 97)),     # 3 bands of rows, ragged last strip
    (24, 24, 6, False, (2, 33, 57)),
    (24, 16, 6, True, (1, 64, 64)),      # no residual (cout != cin)
    (24, 24, 6, False, (1, 5, 7)),       # smaller than one strip and one band
    (24, 24, 6, False, (1, 40, 60)),     # W % 4 == 0 (8-byte output pieces), residual, 4-column last strip
]


@pytest.mark.parametrize("case", FUSED_CASES)
def test_fused_pair_matches_unfused(case, hip_device, monkeypatch):
    """The fused block pair (pool-only pass, SE fold, expand + depthwise recomputed with the gated
    pw-linear conv in the kernel: no hidden-width tensor in HBM) is bit-identical to the
    expand_dw -> se_fold -> pw chain, and within the bf16 bar of the oracle (mobilenetv2.py:153-165)."""
    from arbitrarystyletransfer_amd import mobilenetv2 as M
    inp, oup, t, norm, (n, h, w) = case
    blk = synth.live_init_(DepthWiseConv(inp, oup, 1, t, kernel_size=3, use_norm=norm), 970 + inp + oup)
    blk = blk.eval().to(hip_device).to(torch.bfloat16)
    assert blk._fused_ok(torch.bfloat16, inp, (inp + 15) // 16 * 16, blk.hidden_dim, oup, 3, 1, h, w)
    x = torch.from_numpy(synth.image(971 + inp, (n, inp, h, w)) * 2 - 0.7).to(hip_device).to(torch.bfloat16)
    with torch.no_grad():
        monkeypatch.setattr(M, "FUSED_PAIR", True)
        y_f = blk(x)
        monkeypatch.setattr(M, "FUSED_PAIR", False)
        y_u = blk(x)
        ref = R.mb_block(x.float().cpu(), cpu_sd(blk), "", inp, oup, 1, t, 3, norm, True)
    torch.cuda.synchronize()
    assert torch.equal(y_f, y_u), rel_inf(y_f, y_u)
    assert rel_inf(y_f, ref) <= BF16_BLOCK_TOL


@pytest.mark.parametrize("norm,k", [(True, 3), (True, 5), (False, 3)])
def test_plan_fold_kernel_matches_torch_fold(norm, k, hip_device):
    """The block plan's BatchNorm fold (ast_mb_fold_bn_f32, one launch per conv) is bit-identical to
    the torch expression it replaces (DepthWiseConv._fold: add, sqrt, div, mul, mul, sub), with
    non-trivial running statistics, and zero in the padding of the expand weights."""
    blk = synth.live_init_(DepthWiseConv(20, 24, 1, 6, kernel_size=k, use_norm=norm), 990 + k)
    g = torch.Generator().manual_seed(3)
    with torch.no_grad():
        for m in blk.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.copy_(torch.randn(m.num_features, generator=g))
                m.running_var.copy_(torch.rand(m.num_features, generator=g) * 2 + 0.05)
                m.weight.copy_(torch.randn(m.num_features, generator=g))
                m.bias.copy_(torch.randn(m.num_features, generator=g))
    blk = blk.eval().to(hip_device)
    p = blk._plan(torch.float32, hip_device)
    convs = [i for i, m in enumerate(blk._layers) if isinstance(m, torch.nn.Conv2d)]
    hid = blk.hidden_dim
    w1, b1 = blk._fold(convs[0])
    assert torch.equal(p.w1p[:hid, :20], w1.view(hid, 20))
    assert torch.count_nonzero(p.w1p[:, 20:]) == 0 and torch.count_nonzero(p.w1p[hid:]) == 0
    wd, bd = blk._fold(convs[1])
    assert torch.equal(p.wd, wd.reshape(hid, -1))
    w2, b2 = blk._fold(convs[2])
    assert torch.equal(p.w2, w2.view(24, hid))
    if norm:
        assert torch.equal(p.b1, b1) and torch.equal(p.bd, bd) and torch.equal(p.b2, b2)
    else:
        assert torch.count_nonzero(p.b1) == 0 and torch.count_nonzero(p.bd) == 0 and p.b2 is None


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_ada_out_split_input_matches_cat(dtype, hip_device):
    blk = synth.live_init_(DepthWiseConv(256, 128, 1, 3, use_norm=False, use_identity=False), 7)
    blk = blk.eval().to(hip_device).to(dtype)
    a = torch.from_numpy(synth.image(31, (2, 128, 8, 12))).to(hip_device).to(dtype)
    b = torch.from_numpy(synth.image(32, (2, 128, 8, 12)) - 0.5).to(hip_device).to(dtype)
    with torch.no_grad():
        y_split = blk(a, b)
        y_cat = blk(torch.cat((a, b), 1))
        ref = R.mb_ada_out(a.float().cpu(), b.float().cpu(), cpu_sd(blk))
    torch.cuda.synchronize()
    # the SE pool sums are float atomics (order-dependent in the last bits), so not bitwise
    assert rel_inf(y_split, y_cat) <= (1e-6 if dtype == torch.float32 else 1e-2)
    assert rel_inf(y_split, ref) <= (BLOCK_TOL if dtype == torch.float32 else BF16_BLOCK_TOL)


@pytest.mark.parametrize("xshape,fshape", [((2, 3, 17, 30), (2, 16, 9, 14)),    # 4-pixel kernel
                                           ((2, 3, 13, 40), (2, 16, 7, 32))])   # 8-pixel kernel
def test_dense_convs(xshape, fshape, hip_device):
    enc = synth.live_init_(models.Encoder(), 5).eval().to(hip_device)
    dec = synth.live_init_(models.Decoder(), 6).eval().to(hip_device)
    x = torch.from_numpy(synth.image(41, xshape))
    f = torch.from_numpy(synth.image(42, fshape) - 0.5)
    with torch.no_grad():
        y0 = enc.mob_net[0](x.to(hip_device))
        ref0 = F.hardswish(F.conv2d(F.pad(x, (1, 1, 1, 1), mode="reflect"), enc.mob_net[0][0].weight.cpu()))
        y1 = dec._image_conv(f.to(hip_device))
        w, b = dec._img_out.weight.cpu(), dec._img_out.bias.cpu()
        ref1 = F.conv2d(F.pad(f, (1, 1, 1, 1), mode="reflect"), w, b)
        dec.exporting = True
        y2 = dec._image_conv(f.to(hip_device))
    assert rel_inf(y0, ref0) <= BLOCK_TOL
    assert rel_inf(y1, ref1) <= BLOCK_TOL
    assert rel_inf(y2, F.hardtanh(ref1, 0.0, 1.0)) <= BLOCK_TOL


def _nets(dev, dtype=torch.float32, exporting=True):
    ast = models.AST(exporting=exporting).load_live_init().eval().to(dev).to(dtype)
    enc = synth.live_init_(models.Encoder(), 5).eval()
    dec = synth.live_init_(models.Decoder(), 6).eval()
    ada = synth.live_init_(models.AutoEncoder().ada_out, 7).eval()
    if dtype != torch.float32:   # the oracle runs in fp32 on the same (rounded) weights
        for m in (enc, dec, ada):
            m.to(dtype).float()
    return ast, enc.state_dict(), dec.state_dict(), ada.state_dict()


def _inputs(g):
    shape = tuple(int(s) for s in g["shape"])
    return (torch.from_numpy(synth.image(int(g["seeds"][0]), shape)),
            torch.from_numpy(synth.image(int(g["seeds"][1]), shape)))


@pytest.mark.parametrize("name", ["mb_path_64", "mb_path_128x96"])
def test_encoder_golden(name, golden, hip_device):
    g = golden(name)
    c, _ = _inputs(g)
    ast, *_ = _nets(hip_device)
    with torch.no_grad():
        blocks = ast._enc(c.to(hip_device), out_layers=list(range(15)))
    for i, b in enumerate(blocks):
        cs = b.double().sum(dim=(2, 3)).cpu().numpy()
        ref = g[f"enc_block{i}_chsum"]
        assert np.max(np.abs(cs - ref)) <= CHAIN_TOL * np.abs(ref).max() + 1e-6 * b[0, 0].numel(), i
    assert rel_inf(blocks[12], g["enc12"]) <= CHAIN_TOL
    assert rel_inf(blocks[14], g["enc14"]) <= CHAIN_TOL


@pytest.mark.parametrize("name", ["mb_path_64", "mb_path_128x96"])
def test_decoder_blocks_golden(name, golden, hip_device):
    g = golden(name)
    ast, *_ = _nets(hip_device)
    h = torch.from_numpy(g["t"]).to(hip_device)
    with torch.no_grad():
        for i, block in enumerate(ast._dec._decoder_blocks):
            h = block(h)
            if f"dec_block{i}" in g:
                ref = g[f"dec_block{i}"]
                got = h
                while got.shape != ref.shape:
                    got = got[:, :, ::2, ::2]
                assert rel_inf(got, ref) <= CHAIN_TOL, i
        y = ast._dec._image_conv(h)
    assert rel_inf(y, g["out_export"]) <= CHAIN_TOL


@pytest.mark.parametrize("name", ["mb_path_64", "mb_path_128x96"])
def test_style_transfer_golden(name, golden, hip_device):
    g = golden(name)
    c, s = _inputs(g)
    ast, *_ = _nets(hip_device, exporting=True)
    with torch.no_grad():
        y = ast(c.to(hip_device), s.to(hip_device))
    assert rel_inf(y, g["out_export"]) <= E2E_TOL
    ast2, _, dec_sd, ada_sd = _nets(hip_device, exporting=False)
    with torch.no_grad():
        t_cs, t_return, org_out = ast2(c.to(hip_device), s.to(hip_device))
        org_ref = R.mb_decoder(R.mb_ada_out(torch.from_numpy(g["enc12"]), torch.from_numpy(g["enc14"]), ada_sd), dec_sd)
    assert rel_inf(t_cs, g["out"]) <= E2E_TOL
    assert isinstance(t_return, tuple) and len(t_return) == 2   # the per-layer stylised maps (layers 12, 14)
    if "adain12" in g:
        assert rel_inf(t_return[0], g["adain12"]) <= CHAIN_TOL
        assert rel_inf(t_return[1], g["adain14"]) <= CHAIN_TOL
    assert rel_inf(org_out, org_ref) <= E2E_TOL


def test_autoencoder_vs_oracle(hip_device):
    ae = models.AutoEncoder().load_live_init().eval().to(hip_device)
    x = torch.from_numpy(synth.image(55, (1, 3, 48, 64)))
    _, enc_sd, dec_sd, ada_sd = _nets(hip_device)
    with torch.no_grad():
        y = ae(x.to(hip_device))
        e = R.mb_encoder(x, enc_sd)
        ref = R.mb_decoder(R.mb_ada_out(e[0], e[1], ada_sd), dec_sd)
    assert rel_inf(y, ref) <= E2E_TOL


def check_bf16_segments(ast, c, s, enc_sd, dec_sd, ada_sd, dev):
    """bf16 HIP path vs the fp32 oracle, segment by segment (each segment fed the oracle's input
    rounded to bf16): encoder chain, per-layer AdaIN, ada_out, decoder chain, image conv. The
    end-to-end t is only bounded loosely: AdaIN divides by the content std (down to ~4e-3 at
    layer 12), which amplifies the encoder's bf16 rounding (scripts/mb_bf16_errors.py)."""
    bf = torch.bfloat16
    d = lambda x: x.to(dev).to(bf)  # noqa: E731
    with torch.no_grad():
        cr, sr = R.mb_encoder(c, enc_sd), R.mb_encoder(s, enc_sd)
        ce = ast._enc(d(c), out_layers=[12, 14])
        assert rel_inf(ce[0], cr[0]) <= BF16_CHAIN_TOL and rel_inf(ce[1], cr[1]) <= BF16_CHAIN_TOL
        ar = [R.adain(cr[i].bfloat16().float(), sr[i].bfloat16().float()) for i in range(2)]
        for i in range(2):
            assert rel_inf(ast._adain(d(cr[i]), d(sr[i])), ar[i]) <= BF16_BLOCK_TOL
        tr = R.mb_ada_out(ar[0].bfloat16().float(), ar[1].bfloat16().float(), ada_sd)
        assert rel_inf(ast.ada_out(d(ar[0]), d(ar[1])), tr) <= BF16_BLOCK_TOL
        yr, blocks = R.mb_decoder(tr, dec_sd, exporting=True, return_blocks=True)
        h = d(tr)
        for i, block in enumerate(ast._dec._decoder_blocks):
            h = block(h)
            assert rel_inf(h, blocks[i]) <= BF16_CHAIN_TOL, i
        assert rel_inf(ast._dec._image_conv(d(blocks[-1])), yr) <= BF16_BLOCK_TOL
        y = ast(d(c), d(s))
        assert torch.isfinite(y.float()).all()
        assert rel_inf(ast.encode(d(c), d(s)), tr) <= BF16_E2E_T_TOL


BF16_E2E_TOL = 2e-2   # bf16 HIP path end to end vs the bf16-storage oracle


def check_bf16_end_to_end(ast, c, s, enc_sd, dec_sd, ada_sd, dev):
    """What the bf16 HIP path actually produces (bench --mode mobilenet) against the oracle that
    rounds to bf16 where the HIP path stores bf16 (R.mb_style_transfer_bf16):
      * the image, end to end: BF16_E2E_TOL;
      * the encoder maps (layers 12, 14 of content and style), end to end: BF16_E2E_TOL;
      * t (the decoder input) from the HIP path's own encoder maps: BF16_E2E_TOL.
    t end to end is ill-conditioned, not inaccurate: AdaIN divides by content stds down to ~4e-3,
    so a one-ulp bf16 flip of an encoder output moves t by several percent. Its bound is stated
    against the same spread between two oracles that differ only in rounding order (the fp32
    oracle rounded to bf16 at the encoder outputs vs the bf16-storage oracle): <= 3x that spread."""
    bf = torch.bfloat16
    with torch.no_grad():
        yr, tr = R.mb_style_transfer_bf16(c, s, enc_sd, dec_sd, ada_sd, exporting=True, return_t=True)
        # AST.forward(exporting) step by step (models.py AST.encode: encoder x2 -> per-layer AdaIN ->
        # ada_out; then the decoder), keeping the encoder maps of this very run
        ce, se = ast._enc(c.to(dev).to(bf), out_layers=[12, 14]), ast._enc(s.to(dev).to(bf), out_layers=[12, 14])
        t = ast.ada_out(*ast.stylize_maps(ce, se))
        y = ast._dec(t)
        cr, sr = R.mb_encoder_bf16(c, enc_sd), R.mb_encoder_bf16(s, enc_sd)
        e_enc = max(rel_inf(a, b) for a, b in zip(ce + se, cr + sr))
        t_own = R.mb_block_bf16(torch.cat([R.bf16(R.adain(ce[i].float().cpu(), se[i].float().cpu())) for i in range(2)], 1),
                                ada_sd, "", 256, 128, 1, 3, 3, use_norm=False, use_identity=False)
        c32, s32 = R.mb_encoder(c, enc_sd), R.mb_encoder(s, enc_sd)
        t_alt = R.mb_block_bf16(torch.cat([R.bf16(R.adain(R.bf16(c32[i]), R.bf16(s32[i]))) for i in range(2)], 1),
                                ada_sd, "", 256, 128, 1, 3, 3, use_norm=False, use_identity=False)
    ey, et_own, et, spread = rel_inf(y, yr), rel_inf(t, t_own), rel_inf(t, tr), rel_inf(t_alt, tr)
    print(f"bf16 vs bf16-storage oracle: image {ey:.2e}, encoder maps {e_enc:.2e}, t from own maps {et_own:.2e}, "
          f"t end to end {et:.2e} (oracle-vs-oracle spread {spread:.2e})")
    assert ey <= BF16_E2E_TOL and e_enc <= BF16_E2E_TOL and et_own <= BF16_E2E_TOL, (ey, e_enc, et_own)
    assert et <= max(BF16_E2E_TOL, 3 * spread), (et, spread)


@pytest.mark.parametrize("name", ["mb_path_64", "mb_path_128x96"])
def test_bf16_end_to_end(name, golden, hip_device):
    g = golden(name)
    c, s = _inputs(g)
    ast, enc_sd, dec_sd, ada_sd = _nets(hip_device, torch.bfloat16)
    check_bf16_end_to_end(ast, c, s, enc_sd, dec_sd, ada_sd, hip_device)


def test_bf16_path_64(golden, hip_device):
    g = golden("mb_path_64")
    c, s = _inputs(g)
    ast, enc_sd, dec_sd, ada_sd = _nets(hip_device, torch.bfloat16)
    check_bf16_segments(ast, c.bfloat16().float(), s.bfloat16().float(), enc_sd, dec_sd, ada_sd, hip_device)


def test_config5_shape_bf16_1024(hip_device):
    """Config 5 geometry (1024^2, bf16): one image against the fp32 oracle, plus a B=2 run whose
    images match the B=1 runs (batch independence)."""
    c = torch.from_numpy(synth.image(821, (2, 3, 1024, 1024))).bfloat16()
    s = torch.from_numpy(synth.image(822, (2, 3, 1024, 1024))).bfloat16()
    ast, enc_sd, dec_sd, ada_sd = _nets(hip_device, torch.bfloat16)
    torch.set_num_threads(16)
    check_bf16_segments(ast, c[1:].float(), s[1:].float(), enc_sd, dec_sd, ada_sd, hip_device)
    check_bf16_end_to_end(ast, c.float(), s.float(), enc_sd, dec_sd, ada_sd, hip_device)
    with torch.no_grad():
        y2 = ast(c.to(hip_device), s.to(hip_device))
        y1 = ast(c[1:].to(hip_device), s[1:].to(hip_device))
    assert y2.shape == (2, 3, 1024, 1024)
    # batch independence, bitwise: every reduction is per image and in a fixed order (no atomics)
    assert torch.equal(y2[1:], y1), rel_inf(y2[1:], y1)


def test_mode_dispatch_guards(hip_device):
    blk = DepthWiseConv(16, 16, 1, 6, use_norm=True).to(hip_device)
    x = torch.rand(2, 16, 8, 8, device=hip_device)
    with torch.no_grad():
        assert blk(x).shape == (2, 16, 8, 8)   # training mode: the batch-statistics kernels (mbtrain)
    bns = [m for m in blk.modules() if isinstance(m, torch.nn.BatchNorm2d)]
    assert bns and all(int(m.num_batches_tracked) == 1 for m in bns)
    blk.eval()
    with pytest.raises(NotImplementedError):
        blk(x)                          # eval-mode BatchNorm under autograd recording
    with torch.no_grad():
        assert blk(x).shape == (2, 16, 8, 8)
