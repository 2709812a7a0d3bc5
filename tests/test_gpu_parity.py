"""GPU parity: every HIP kernel on the hot path against the CPU oracle (oracle/ref_cpu.py) on the
same seeded inputs, and against the golden vectors produced by the reference's own code.

Tolerances (fp32): single ops rel_inf <= 2e-5; the 18-conv encoder->AdaIN->decoder path
rel_inf = max|a-b|/max|b| <= 1e-3 (north-star bar) and elementwise |a-b| <= 1e-3*(|b|+max|b|).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from arbitrarystyletransfer_amd import models, ops, synth
from arbitrarystyletransfer_amd._lib import lib
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu

E2E_TOL = 1e-3
OP_TOL = 2e-5


def rel_inf(a, b):
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


def assert_e2e(a, b):
    a = np.asarray(a.detach().cpu(), np.float64)
    b = np.asarray(b, np.float64)
    assert rel_inf(a, b) <= E2E_TOL, rel_inf(a, b)
    assert np.all(np.abs(a - b) <= E2E_TOL * (np.abs(b) + np.max(np.abs(b))))


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def oracle_conv(x, w, b, up, pad_mode, normalize, relu):
    if normalize:
        x = R.normalization(x)
    if up == 2:
        x = F.interpolate(x, scale_factor=2, mode="nearest")
    if pad_mode == "reflect":
        y = F.conv2d(F.pad(x, (1, 1, 1, 1), mode="reflect"), w, b)
    else:
        y = F.conv2d(x, w, b, padding=1)
    return y, F.relu(y), F.max_pool2d(F.relu(y), 2, 2) if y.shape[2] >= 2 and y.shape[3] >= 2 else None


CONV_CASES = [
    # n, cin, h, w, cout, up, pad, normalize
    (2, 3, 17, 40, 64, 1, "zeros", True),     # conv_1 shape class, ragged H, 2 x-tiles
    (1, 16, 64, 64, 128, 1, "zeros", False),
    (2, 24, 8, 12, 64, 1, "reflect", False),  # W < tile width, W % 4 == 0
    (1, 32, 16, 16, 128, 2, "reflect", False),  # upsample
    (2, 8, 5, 7, 64, 2, "reflect", False),    # odd sizes + upsample
    (1, 64, 32, 96, 3, 1, "reflect", False),  # final decoder conv (cout 3)
    (1, 12, 6, 10, 64, 1, "reflect", False),  # W % 4 != 0: scalar gather path
    (1, 40, 33, 64, 64, 1, "zeros", False),   # odd H, cin not a multiple of the K chunk
    (1, 3, 9, 130, 16, 1, "reflect", False),  # cin 3, cout 16 (MobileNet block 0 class), W % 4 != 0, 2 x-tiles
    (2, 4, 12, 64, 24, 1, "zeros", False),   # cin 4, cout 24
    (1, 1, 5, 36, 64, 1, "reflect", False),   # cin 1 (zero channels of the 4-channel template)
    # cin 1 / 2 on the direct kernel with wide weight slabs: its LDS holds the CIN = 4 template's
    # 4 x 9 x cout_pad weights (sized by Cin before round 4, which read past the allocation)
    (1, 2, 10, 70, 128, 1, "zeros", False),
    (2, 1, 9, 128, 192, 1, "reflect", False),
    (2, 3, 16, 256, 64, 1, "zeros", True),    # conv_1: full 128-px tiles, normalised gather
    (1, 18, 8, 256, 3, 1, "reflect", False),  # cout 3, vector-staged tiles, partial last K chunk
    (1, 10, 6, 128, 4, 2, "reflect", False),  # cout 4, upsampled, vector-staged tiles
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv3x3_all_configs(case, hip_device):
    n, cin, h, w, cout, up, pad, norm = case
    x = torch.from_numpy(synth.image(100 + cin, (n, cin, h, w)) * 2 - 0.5)
    wt = torch.from_numpy(synth.conv_weight(200 + cin, cout, cin, 3))
    bs = torch.from_numpy(synth.conv_bias(300 + cin, cout))
    pre_r, act_r, pool_r = oracle_conv(x, wt, bs, up, pad, norm, True)
    xd, wp, bd = x.to(hip_device), ops.pack_conv3x3(wt.to(hip_device)), bs.to(hip_device)
    mean = torch.tensor(R.IMNET_MEAN, device=hip_device) if norm else None
    std = torch.tensor(R.IMNET_STD, device=hip_device) if norm else None
    ncfg = lib().ast_conv3x3_num_configs()
    tried = 0
    for cfg in range(ncfg):
        try:
            pre, act, pool = ops.conv3x3(xd, wp, bd, cout, upsample=up, pad_mode=pad, in_mean=mean, in_std=std,
                                         want_pre=True, want_act=True, want_pool=pool_r is not None, cfg=cfg)
        except Exception as e:  # configurations that do not support this cout are rejected on the host
            assert "unsupported" in str(e), e
            continue
        tried += 1
        torch.cuda.synchronize()
        assert rel_inf(pre, pre_r) <= OP_TOL, (cfg, rel_inf(pre, pre_r))
        assert rel_inf(act, act_r) <= OP_TOL, cfg
        if pool_r is not None:
            assert rel_inf(pool, pool_r) <= OP_TOL, cfg
    assert tried >= 1


PERSIST_CASES = [
    # n, cin, h, w, cout, up, pad, pool: several blocks per workgroup slot for every config 32-35
    (4, 40, 130, 200, 192, 1, "zeros", True),   # partial last K chunk, ragged tiles, 3 channel groups
    (8, 32, 64, 100, 64, 2, "reflect", False),  # upsampled
    (3, 64, 66, 72, 128, 1, "reflect", True),   # blocks per slot not a whole number
]


@pytest.mark.parametrize("case", PERSIST_CASES)
def test_conv3x3_persistent_bit_identical(case, hip_device):
    """Configs 32-35 (one workgroup per CU slot walking its blocks, next block's first chunk loaded
    under the current epilogue) and 38-41 (the round-5 block loop around the same block code)
    against their one-block-per-workgroup forms 28-31: same k order and rounding per block, so the
    outputs are bit-identical, and repeated launches agree."""
    n, cin, h, w, cout, up, pad, pool = case
    x = torch.from_numpy(synth.image(700 + cin, (n, cin, h, w)) * 2 - 0.5).to(hip_device)
    wt = torch.from_numpy(synth.conv_weight(710 + cin, cout, cin, 3)).to(hip_device)
    bd = torch.from_numpy(synth.conv_bias(720 + cin, cout)).to(hip_device)
    wp = ops.pack_conv3x3(wt)
    for cfg in (28, 29, 30, 31):
        ref = ops.conv3x3(x, wp, bd, cout, upsample=up, pad_mode=pad, want_pre=True, want_act=True, want_pool=pool,
                          cfg=cfg)
        for pc in (cfg + 4, cfg + 4, cfg + 10, cfg + 10):
            got = ops.conv3x3(x, wp, bd, cout, upsample=up, pad_mode=pad, want_pre=True, want_act=True,
                              want_pool=pool, cfg=pc)
            torch.cuda.synchronize()
            for r, g in zip(ref, got):
                if r is not None:
                    assert torch.equal(r, g), (pc, (r - g).abs().max().item())


POOL_ONLY_CASES = [
    # n, cin, h, w, cout, pad: the encoder's pool layers, ragged tiles, W/2 % 4 != 0, partial channel tiles
    (2, 64, 32, 64, 64, "zeros"),
    (1, 40, 18, 70, 48, "zeros"),
    (3, 128, 17, 36, 128, "reflect"),
    (1, 16, 6, 10, 24, "zeros"),
]


@pytest.mark.parametrize("case", POOL_ONLY_CASES)
def test_conv3x3_pool_only_bit_identical(case, hip_device):
    """ReLU + max-pool as the only output (config 2's encoder pool layers): the split-bf16 M16 kernels
    pool in registers (no LDS staging); the pooled map must equal, bit for bit, the pool the same
    configuration writes beside the pre-ReLU and ReLU maps (the staged path), and the oracle."""
    n, cin, h, w, cout, pad = case
    x = torch.from_numpy(synth.image(81 + cin, (n, cin, h, w)) * 2 - 0.5)
    wt = torch.from_numpy(synth.conv_weight(82, cout, cin, 3))
    bs = torch.from_numpy(synth.conv_bias(83, cout))
    _, _, pool_r = oracle_conv(x, wt, bs, 1, pad, False, True)
    xd, wp, bd = x.to(hip_device), ops.pack_conv3x3(wt.to(hip_device)), bs.to(hip_device)
    for cfg in (-1, 28, 29, 30, 31, 38, 39, 40, 41):
        try:
            _, _, p_only = ops.conv3x3(xd, wp, bd, cout, pad_mode=pad, want_pre=False, want_act=False,
                                       want_pool=True, cfg=cfg)
            _, _, p_all = ops.conv3x3(xd, wp, bd, cout, pad_mode=pad, want_pre=True, want_act=True, want_pool=True,
                                      cfg=cfg)
        except Exception as e:
            assert "unsupported" in str(e), e
            continue
        torch.cuda.synchronize()
        assert torch.equal(p_only, p_all), (cfg, float((p_only - p_all).abs().max()))
        assert rel_inf(p_only, pool_r) <= OP_TOL, (cfg, rel_inf(p_only, pool_r))


@pytest.mark.parametrize("cin", [1, 2, 3, 4])
def test_conv3x3_direct_cin_le4_lds_weights(cin, hip_device):
    """The direct cin <= 4 kernel (configs 18-23) on every cin it takes, with a 192-channel weight
    slab (27.6 KB of LDS for the 4-channel template): launched explicitly, never rejected."""
    x = torch.from_numpy(synth.image(40 + cin, (2, cin, 12, 136)) * 2 - 0.5)
    wt = torch.from_numpy(synth.conv_weight(50 + cin, 192, cin, 3))
    bs = torch.from_numpy(synth.conv_bias(60 + cin, 192))
    pre_r, act_r, _ = oracle_conv(x, wt, bs, 1, "reflect", False, True)
    xd, wp, bd = x.to(hip_device), ops.pack_conv3x3(wt.to(hip_device)), bs.to(hip_device)
    for cfg in range(18, 24):
        pre, act, _ = ops.conv3x3(xd, wp, bd, 192, pad_mode="reflect", want_pre=True, want_act=True, cfg=cfg)
        torch.cuda.synchronize()
        assert rel_inf(pre, pre_r) <= OP_TOL, (cin, cfg, rel_inf(pre, pre_r))
        assert rel_inf(act, act_r) <= OP_TOL, (cin, cfg)


def test_conv3x3_pair_input_matches_concat(hip_device):
    x1 = torch.from_numpy(synth.image(1, (2, 16, 24, 64))).to(hip_device)
    x2 = torch.from_numpy(synth.image(2, (3, 16, 24, 64))).to(hip_device)
    wt = torch.from_numpy(synth.conv_weight(3, 64, 16, 3)).to(hip_device)
    wp = ops.pack_conv3x3(wt)
    _, a, _ = ops.conv3x3(x1, wp, None, 64, x2=x2)
    _, b, _ = ops.conv3x3(torch.cat([x1, x2]), wp, None, 64)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_conv3x3_nan_propagates(hip_device):
    x = torch.ones(1, 8, 8, 32)
    x[0, 3, 4, 5] = float("nan")
    wt = torch.from_numpy(synth.conv_weight(5, 64, 8, 3))
    pre_r, act_r, pool_r = oracle_conv(x, wt, None, 1, "zeros", False, True)
    pre, act, pool = ops.conv3x3(x.to(hip_device), ops.pack_conv3x3(wt.to(hip_device)), None, 64,
                                 want_pre=True, want_act=True, want_pool=True)
    for got, ref in ((pre, pre_r), (act, act_r), (pool, pool_r)):
        g = got.cpu().numpy()
        r = ref.numpy()
        np.testing.assert_array_equal(np.isnan(g), np.isnan(r))


def test_conv3x3_split_bf16_nonfinite_and_overflow(hip_device):
    """The split-bf16 kernel's contract for extreme inputs (csrc/conv3x3_igemm.hip split3):
    * a finite input above bf16's largest value (3.3895e38) is split exactly (hi clamped), so a
      single large pixel gives the same output as torch, to fp32 accuracy;
    * an inf input gives a non-finite value at every output it reaches: +-inf with torch's sign,
      or NaN where the MFMA's inf * (the weight's mid / lo term = 0) product occurs (torch gives
      +-inf there); all other outputs are unchanged. A NaN input gives NaN where torch does
      (test_conv3x3_nan_propagates)."""
    n, cin, h, w, cout = 1, 64, 16, 32, 64
    wt = torch.from_numpy(synth.conv_weight(41, cout, cin, 3)) * 0.01
    wp = ops.pack_conv3x3(wt.to(hip_device))
    x = torch.zeros(n, cin, h, w)
    x[0, 7, 5, 9] = 3.4e38
    ref, _, _ = oracle_conv(x.double(), wt.double(), None, 1, "zeros", False, False)
    got, _, _ = ops.conv3x3(x.to(hip_device), wp, None, cout, want_pre=True, want_act=False)
    assert torch.isfinite(got).all()
    assert rel_inf(got, ref.float()) <= 2e-6
    x = torch.from_numpy(synth.image(42, (n, cin, h, w)))
    x[0, 7, 5, 9] = float("inf")
    ref, _, _ = oracle_conv(x, wt, None, 1, "zeros", False, False)
    got, _, _ = ops.conv3x3(x.to(hip_device), wp, None, cout, want_pre=True, want_act=False)
    g, r = got.cpu().numpy(), ref.numpy()
    touched = ~np.isfinite(r)
    assert touched.sum() == cout * 9
    assert not np.isfinite(g[touched]).any()
    inf = np.isinf(g) & touched
    assert np.array_equal(np.sign(g[inf]), np.sign(r[inf]))
    assert np.allclose(g[~touched], r[~touched], rtol=1e-5, atol=1e-5 * np.abs(r[~touched]).max())


def test_adain_golden(golden, hip_device):
    g = golden("adain_kat")
    c, s = T(g["content"], hip_device), T(g["style"], hip_device)
    assert rel_inf(ops.adain(c, s), g["out"]) <= OP_TOL
    assert rel_inf(ops.adain(c, s, swap_style_stats=False), g["out_canonical"]) <= OP_TOL
    assert rel_inf(models.AdaIN()(c, s), g["out"]) <= OP_TOL
    z = ops.adain(T(g["content_zerovar"], hip_device), s).cpu().numpy()
    np.testing.assert_array_equal(np.isnan(z), np.isnan(g["out_zerovar"]))
    m = ~np.isnan(g["out_zerovar"])
    assert np.max(np.abs(z[m] - g["out_zerovar"][m])) <= OP_TOL * np.max(np.abs(g["out_zerovar"][m]))


@pytest.mark.parametrize("shape,alpha", [((2, 64, 64, 64), 1.0), ((1, 512, 8, 8), 0.3), ((3, 7, 5, 9), 0.5),
                                         ((1, 4, 1, 1), 1.0)])
def test_adain_vs_oracle(shape, alpha, hip_device):
    c = torch.from_numpy(synth.image(11, shape) * 3)
    s = torch.from_numpy(synth.image(12, shape) * 2 + 1)
    ref = R.alpha_blend(R.adain(c, s), c, alpha)
    got = ops.adain(c.to(hip_device), s.to(hip_device), alpha=alpha).cpu()
    if shape[2] * shape[3] == 1:  # 1x1 maps: unbiased std = 0/0 -> NaN, as in torch
        assert torch.isnan(got).all() and torch.isnan(ref).all()
    else:
        assert rel_inf(got, ref) <= OP_TOL


def test_stats_golden(golden, hip_device):
    g = golden("stats")
    f = T(g["feat"], hip_device)
    m, s = models.channel_stats(f)
    assert rel_inf(m, g["cs_mean"]) <= OP_TOL and rel_inf(s, g["cs_std"]) <= OP_TOL
    m2, s2 = models.calc_mean_std(f)
    assert rel_inf(m2, g["cms_mean"]) <= OP_TOL and rel_inf(s2, g["cms_std"]) <= OP_TOL
    assert rel_inf(models.mean_variance_norm(f), g["mvn"]) <= OP_TOL


def test_encoder_relu4_1_golden(golden, hip_device):
    g = golden("vgg_path_64")
    enc = models.PretrainedEncoder(["relu_9"]).to(hip_device)
    fc = enc(T(g["content"], hip_device))
    assert len(fc) == 1
    assert rel_inf(fc[0], g["relu4_1_content"]) <= 1e-4
    both = enc(T(g["content"], hip_device), T(g["style"], hip_device))[0]
    assert rel_inf(both[1:], g["relu4_1_style"]) <= 1e-4


def test_lossnet_layers_golden(golden, hip_device):
    g = golden("lossnet_32")
    enc = models.PretrainedEncoder().to(hip_device)
    maps = enc(T(g["x"], hip_device))
    names = ["conv_1", "conv_3", "conv_5", "conv_9", "conv_13", "relu_15"]
    assert len(maps) == len(names)
    for n, m in zip(names, maps):
        assert rel_inf(m, g[n]) <= 1e-4, n


def test_decoder_golden(golden, hip_device):
    g = golden("decoder_6x10")
    dec = models.VGGDecoder().to(hip_device)
    assert_e2e(dec(T(g["t"], hip_device)), g["out"])


@pytest.mark.parametrize("name", ["vgg_path_64", "vgg_path_128"])
def test_style_transfer_golden(name, golden, hip_device):
    g = golden(name)
    net = models.AdaINStyleTransfer().to(hip_device)
    y = net(T(g["content"], hip_device), T(g["style"], hip_device))
    assert_e2e(y, g["out"])
    if "out_alpha_half" in g:
        assert_e2e(net(T(g["content"], hip_device), T(g["style"], hip_device), alpha=0.5), g["out_alpha_half"])


def test_style_transfer_256_config1(golden, hip_device):
    g = golden("vgg_path_256_summary")
    net = models.AdaINStyleTransfer().to(hip_device)
    c = torch.from_numpy(synth.image(797, (1, 3, 256, 256))).to(hip_device)
    s = torch.from_numpy(synth.image(798, (1, 3, 256, 256))).to(hip_device)
    with torch.no_grad():
        y = net(c, s)
    assert_e2e(y[:, :, ::4, ::4], g["sub4"])
    cs = y.double().sum(dim=(2, 3)).cpu().numpy()
    np.testing.assert_allclose(cs, g["chan_sum"], rtol=1e-3, atol=1e-3 * np.abs(g["chan_sum"]).max())


def test_style_transfer_512_batch8_vs_oracle(hip_device):
    """Bench configuration (config 2: B=8, 512^2): images 0 and 7 checked against the CPU oracle."""
    c = synth.image(777, (8, 3, 512, 512))
    s = synth.image(778, (8, 3, 512, 512))
    net = models.AdaINStyleTransfer().to(hip_device)
    with torch.no_grad():
        y = net(torch.from_numpy(c).to(hip_device), torch.from_numpy(s).to(hip_device)).cpu()
    enc = [(torch.from_numpy(w), torch.from_numpy(b)) for w, b in synth.vgg_encoder_weights(1)[:9]]
    dec = [(torch.from_numpy(w), torch.from_numpy(b)) for w, b in synth.vgg_decoder_weights(2)]
    for i in (0, 7):
        ref = R.style_transfer(torch.from_numpy(c[i:i + 1]), torch.from_numpy(s[i:i + 1]), enc, dec)
        assert_e2e(y[i:i + 1], ref.numpy())
    assert torch.isfinite(y).all()


def test_one_style_many_contents_stats(hip_device):
    """stylize_with_stats (AdaIN from broadcastable style statistics) equals the
    regular forward with the style replicated across the batch, and the kernel matches the oracle."""
    net = models.AdaINStyleTransfer().to(hip_device)
    c = torch.from_numpy(synth.image(931, (3, 3, 64, 96))).to(hip_device)
    s = torch.from_numpy(synth.image(932, (1, 3, 64, 96))).to(hip_device)
    with torch.no_grad():
        m, sd = net.style_statistics(s)
        y = net.stylize_with_stats(c, m[0], sd[0], alpha=0.8)
        ref = net(c, s.expand(3, -1, -1, -1).contiguous(), alpha=0.8)
        fc = net.encoder(c)[0]
        t = ops.adain_stats(fc, m[0], sd[0], alpha=1.0)
        t2 = ops.adain_stats(fc, m.expand(3, -1).contiguous(), sd.expand(3, -1).contiguous(), alpha=1.0)
    assert rel_inf(y, ref) <= OP_TOL * 10
    assert torch.equal(t, t2)
    assert rel_inf(t, R.adain_from_stats(fc.cpu(), m[0].cpu(), sd[0].cpu())) <= OP_TOL


@pytest.mark.parametrize("cin,pad,norm", [(3, "zeros", True), (3, "reflect", False), (4, "zeros", False)])
def test_conv3x3_direct_cin4_matches_mfma(cin, pad, norm, hip_device):
    """The direct cin <= 4 kernel (cfg 20) accumulates in the fp32 MFMA kernel's order (tap-major,
    channel-minor fmaf chain), so the two give the same bits. (Since round 6 conv_1 runs the
    split-bf16 cfg 42 by default; the ReLU / max-pool routing the training-step oracle tests use is
    read from the GPU forward itself, so it follows whichever kernel runs.)"""
    x = torch.from_numpy(synth.image(31 + cin, (2, cin, 24, 160))).to(hip_device)
    wt = torch.from_numpy(synth.conv_weight(32, 64, cin, 3)).to(hip_device)
    b = torch.from_numpy(synth.conv_bias(33, 64)).to(hip_device)
    wp = ops.pack_conv3x3(wt)
    mean = torch.tensor(R.IMNET_MEAN, device=hip_device)[:cin] if norm else None
    std = torch.tensor(R.IMNET_STD, device=hip_device)[:cin] if norm else None
    kw = dict(pad_mode=pad, in_mean=mean, in_std=std, want_pre=True, want_act=True)
    p20, a20, _ = ops.conv3x3(x, wp, b, 64, cfg=20, **kw)
    p7, a7, _ = ops.conv3x3(x, wp, b, 64, cfg=7, **kw)
    torch.cuda.synchronize()
    assert torch.equal(p20, p7), float((p20 - p7).abs().max())
    assert torch.equal(a20, a7)


CIN3_CASES = [
    # n, cin, h, w, cout, pad, norm, n2 (second batch of the pair input)
    (2, 3, 37, 150, 64, "zeros", True, 1),    # conv_1: ragged 16-row and 64-column tiles, content|style pair
    (1, 3, 16, 64, 40, "reflect", False, 0),  # cout 40: a partial 16-channel block of the second half
    (1, 2, 9, 70, 130, "zeros", False, 0),    # cin 2, three 64-channel groups, W % 4 != 0
    (3, 1, 5, 3, 16, "reflect", False, 0),    # cin 1, plane narrower than a 32-pixel block
]


@pytest.mark.parametrize("case", CIN3_CASES)
def test_conv3x3_cin3_split_bf16(case, hip_device):
    """The split-bf16 MFMA kernel for cin <= 3 (configurations 42, 43; csrc/conv_cin3.hip) against
    the float64 oracle at the fp32 bar, on ragged tiles, partial channel blocks and the pair input;
    its two tile heights are the same arithmetic per output, so they agree bit for bit."""
    n, cin, h, w, cout, pad, norm, n2 = case
    x = torch.from_numpy(synth.image(61 + cin, (n + n2, cin, h, w)) * 2 - 0.5)
    wt = torch.from_numpy(synth.conv_weight(62, cout, cin, 3))
    bs = torch.from_numpy(synth.conv_bias(63, cout))
    pre_r, act_r, _ = oracle_conv(x, wt, bs, 1, pad, norm, True)
    xd, wp, bd = x.to(hip_device), ops.pack_conv3x3(wt.to(hip_device)), bs.to(hip_device)
    mean = torch.tensor(R.IMNET_MEAN, device=hip_device)[:cin] if norm else None
    std = torch.tensor(R.IMNET_STD, device=hip_device)[:cin] if norm else None
    outs = []
    for cfg in (42, 43):
        pre, act, _ = ops.conv3x3(xd[:n], wp, bd, cout, pad_mode=pad, in_mean=mean, in_std=std, want_pre=True,
                                  want_act=True, cfg=cfg, x2=xd[n:] if n2 else None)
        torch.cuda.synchronize()
        assert rel_inf(pre, pre_r) <= OP_TOL, (cfg, rel_inf(pre, pre_r))
        assert rel_inf(act, act_r) <= OP_TOL, cfg
        outs.append((pre, act))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("parts", ["mask", "all", "none"])
def test_conv3x3_cin3_dgrad_epilogue(parts, hip_device):
    """Input gradient of a 64 -> 3 conv (the decoder's last layer) through configurations 42 / 43:
    the dgrad conv reads the 3 channels of dy; fused ReLU-mask / tap-gradient epilogue against CPU
    autograd; the configurations agree bit for bit with each other."""
    from arbitrarystyletransfer_amd._lib import lib as L, ptr, stream_ptr
    from arbitrarystyletransfer_amd.functional import _TF
    n, cin, H, W = 2, 64, 19, 100
    wt = torch.from_numpy(synth.conv_weight(71, 3, cin, 3))
    dy = torch.from_numpy(synth.image(72, (n, 3, H, W)) * 2 - 1)
    mask = torch.from_numpy(synth.image(73, (n, cin, H, W)) * 2 - 1).clamp_min(0.0)
    ap = torch.from_numpy(synth.image(74, (n, cin, H, W)) * 2 - 1)
    aq = torch.from_numpy(synth.image(75, (n, cin, H, W)) * 2 - 1)
    xr = torch.zeros((n, cin, H, W), requires_grad=True)
    (F.conv2d(F.pad(xr, (1, 1, 1, 1)), wt) * dy).sum().backward()
    g = xr.grad
    if parts == "none":
        mask = ap = aq = None
        ref = g
    elif parts == "mask":
        ap = aq = None
        ref = torch.where(mask > 0, g, torch.zeros_like(g))
    else:
        ref = torch.where(mask > 0, aq + (g + ap), aq)
    d = hip_device
    to = lambda t: None if t is None else t.to(d)  # noqa: E731
    dyd, md, apd, aqd = to(dy), to(mask), to(ap), to(aq)
    wtf = _TF.get(wt.to(d))
    outs = []
    for cfg in (42, 43):
        dx = torch.empty((n, cin, H, W), device=d)
        rc = L().ast_conv3x3_dgrad_f32(cfg, ptr(dyd), ptr(wtf), ptr(dx), ptr(md), ptr(apd), ptr(aqd), n, 3, H, W,
                                       cin, 1, stream_ptr(d))
        assert rc == 0, (cfg, rc)
        torch.cuda.synchronize()
        assert rel_inf(dx, ref) <= OP_TOL * 2.5, (cfg, rel_inf(dx, ref))
        outs.append(dx)
    assert torch.equal(outs[0], outs[1])


def test_torch_ops_equal_ctypes_path(hip_device):
    """torch.ops.ast_hip.* (the dispatcher registration, csrc/torch_ops.cpp) launches the same
    kernels as the ctypes binding: outputs are bit-identical."""
    from arbitrarystyletransfer_amd import ops, torch_ops
    o = torch_ops.load()
    d = hip_device
    c = torch.from_numpy(synth.image(3, (2, 64, 24, 40))).to(d) * 3 + 1
    s = torch.from_numpy(synth.image(4, (2, 64, 17, 9))).to(d) * 2
    for alpha, swap in ((1.0, True), (0.4, False)):
        assert torch.equal(o.adain(c, s, alpha, swap), ops.adain(c, s, alpha=alpha, swap_style_stats=swap))
    for unb, eps in ((True, 0.0), (True, 1e-5), (False, 0.0)):
        a, b = o.channel_stats(c, unb, eps), ops.channel_stats(c, unb, eps)
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    w = torch.from_numpy(synth.conv_weight(5, 128, 64, 3)).to(d)
    bias = torch.from_numpy(synth.conv_bias(6, 128)).to(d)
    pk = o.conv3x3_pack(w)
    assert torch.equal(pk, ops.pack_conv3x3(w))
    for up, pad, pool in ((1, 0, True), (2, 1, False)):
        got = o.conv3x3_fwd(c, pk, bias, 128, up, pad, None, None, True, True, pool, -1)
        ref = ops.conv3x3(c, pk, bias, 128, upsample=up, pad_mode=("zeros", "reflect")[pad], want_pre=True,
                          want_act=True, want_pool=pool, cfg=-1, _pack=False)
        for g, r in zip(got, ref):
            assert (r is None and g.numel() == 0) or torch.equal(g, r)
    img = torch.from_numpy(synth.image(7, (2, 3, 40, 36))).to(d)
    w1 = torch.from_numpy(synth.conv_weight(8, 64, 3, 3)).to(d)
    mean = torch.tensor([0.485, 0.456, 0.406], device=d)
    std = torch.tensor([0.229, 0.224, 0.225], device=d)
    got = o.conv3x3_fwd(img, o.conv3x3_pack(w1), None, 64, 1, 0, mean, std, True, True, False, -1)
    ref = ops.conv3x3(img, ops.pack_conv3x3(w1), None, 64, in_mean=mean, in_std=std, want_pre=True, want_act=True,
                      cfg=-1, _pack=False)
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
    f = torch.from_numpy(synth.image(9, (2, 64, 32, 32))).to(d)
    from arbitrarystyletransfer_amd import losses as L
    g1 = o.gram(f)
    assert torch.equal(g1, L.gram_matrix(f))   # split-K partials summed in split order: same bits


SMALLC_CASES = [
    # n, cin, h, w, cout, pad: the cout <= 4 convs (decoder image conv 64 -> 3, the loss network's
    # conv_1 input gradient 64 -> 3) at tile-ragged sizes
    (1, 64, 32, 96, 3, "reflect"),
    (2, 64, 17, 260, 3, "zeros"),    # ragged H, W not a multiple of the 256-column wave tile
    (1, 18, 8, 512, 4, "reflect"),   # two column tiles, cout 4, cin not a multiple of 4
    (3, 5, 3, 68, 3, "zeros"),       # 3-row maps, 17 quads per row
    (1, 64, 2, 8, 4, "reflect"),     # smallest reflect-padded map
]


@pytest.mark.parametrize("case", SMALLC_CASES)
def test_conv3x3_smallc_streaming_bit_identical(case, hip_device):
    """configs 36 / 37 (register-streaming direct conv, cout <= 4) against the oracle and bit-identical
    to configs 10 / 11 (LDS-staged), which sum every output in the same tap-major, channel-minor order."""
    n, cin, h, w, cout, pad = case
    x = torch.from_numpy(synth.image(400 + cin, (n, cin, h, w)) * 2 - 0.5)
    wt = torch.from_numpy(synth.conv_weight(500 + cin, cout, cin, 3))
    bs = torch.from_numpy(synth.conv_bias(600 + cin, cout))
    pre_r, act_r, _ = oracle_conv(x, wt, bs, 1, pad, False, True)
    xd, wp, bd = x.to(hip_device), ops.pack_conv3x3(wt.to(hip_device)), bs.to(hip_device)
    old = ops.conv3x3(xd, wp, bd, cout, pad_mode=pad, want_pre=True, want_act=True, cfg=10 if cout <= 3 else 11)
    new = ops.conv3x3(xd, wp, bd, cout, pad_mode=pad, want_pre=True, want_act=True, cfg=36 if cout <= 3 else 37)
    assert rel_inf(new[0], pre_r) <= OP_TOL
    assert rel_inf(new[1], act_r) <= OP_TOL
    assert torch.equal(new[0], old[0]) and torch.equal(new[1], old[1])
    # the content|style pair input (x2) of the encoder path
    half = n // 2
    if half:
        pair = ops.conv3x3(xd[:half], wp, bd, cout, pad_mode=pad, want_pre=True, want_act=False, x2=xd[half:],
                           cfg=36 if cout <= 3 else 37)
        assert torch.equal(pair[0], new[0])
