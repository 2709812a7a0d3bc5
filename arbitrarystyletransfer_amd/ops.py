"""Functional wrappers over the HIP kernels (C ABI in include/ast_hip.h).

Each op takes device tensors, checks shapes/dtypes on the host (a kernel is never launched on a
shape it does not support), allocates outputs with the PyTorch caching allocator and enqueues the
kernel on the current HIP stream. No host synchronisation, so sequences of ops can be captured
into a hipGraph. CPU tensors raise: there is no CPU fallback in the product path.
"""
from __future__ import annotations

import os

import torch

from ._lib import HipOpError, check, lib, ptr, stream_ptr

PAD_MODES = {"zeros": 0, "reflect": 1}

# Bumped by optimizers that update parameters through raw pointers (optim.FusedAdam), which
# torch's per-tensor _version counter cannot see; weight-pack caches key on it. Per parameter
# (`_ast_epoch`), so the packs of frozen weights (the VGG loss network) survive optimizer steps.
WEIGHTS_EPOCH = [0]


def bump_weights_epoch(params=None):
    WEIGHTS_EPOCH[0] += 1
    for p in params or ():
        p._ast_epoch = getattr(p, "_ast_epoch", 0) + 1


def weight_epoch(t) -> int:
    """The update count of parameter t by raw-pointer optimizers (cache keys)."""
    return getattr(t, "_ast_epoch", 0)


class LaunchTimer:
    """Records a pair of HIP events around every conv3x3 launch, on the launch stream, while
    active (bench.py's live roofline measurement). Use as a context manager."""

    active = None

    def __init__(self):
        self.records = []  # (tag, flops, start_event, end_event)

    def __enter__(self):
        LaunchTimer.active = self
        return self

    def __exit__(self, *exc):
        LaunchTimer.active = None

    def results(self):
        """[(tag, flops, milliseconds)] — call after synchronising the device."""
        return [(tag, fl, s.elapsed_time(e)) for tag, fl, s, e in self.records]


def _timed(tag, flops, device, launch):
    t = LaunchTimer.active
    if t is None:
        return launch()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    stream = torch.cuda.current_stream(device)
    s.record(stream)
    code = launch()
    e.record(stream)
    t.records.append((tag, flops, s, e))
    return code


def _dev(t: torch.Tensor, name: str) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a tensor")
    if t.device.type != "cuda":
        raise HipOpError(f"{name} is on {t.device}; arbitrarystyletransfer_amd runs on MI355X (HIP) devices only")
    if t.dtype != torch.float32:
        raise HipOpError(f"{name} must be float32, got {t.dtype}")
    return t.contiguous()


# ------------------------------------------------------------------------------------------------
# 3x3 convolution
# ------------------------------------------------------------------------------------------------

_TUNING = None


def tuned_config(n, cin, h_in, w_in, cout, up, pad_mode, pool, kind="") -> int:
    """Kernel configuration measured fastest for this shape (scripts/tune_conv.py writes
    conv_tuning.json); -1 (the library's own heuristic) for shapes never tuned. `kind` separates
    launches of the same GEMM shape with another epilogue (" dgrad": the input-gradient conv of
    ast_conv3x3_dgrad_f32, " dgrad sum2" with its 2x2-sum upsample adjoint), timed on their own."""
    global _TUNING
    if _TUNING is None:
        import json
        import os
        path = os.environ.get("AST_CONV_TUNING") or os.path.join(  # override: A/B of tuning tables
            os.path.dirname(os.path.abspath(__file__)), "conv_tuning.json")
        try:
            with open(path) as f:
                _TUNING = json.load(f)
        except (OSError, ValueError):
            _TUNING = {}
    k = f"{n}x{cin}x{h_in}x{w_in}->{cout} up{up} {pad_mode}{' pool' if pool else ''}{kind}"
    return int(_TUNING.get(k, -1))

def pack_conv3x3(weight: torch.Tensor) -> torch.Tensor:
    """Repack a [cout, cin, 3, 3] filter bank into the kernel's [cin_pad][9][cout_pad] layout."""
    w = _dev(weight, "weight")
    if w.dim() != 4 or w.shape[2:] != (3, 3):
        raise HipOpError(f"conv3x3 weight must be [cout, cin, 3, 3], got {tuple(w.shape)}")
    cout, cin = int(w.shape[0]), int(w.shape[1])
    L = lib()
    out = torch.empty(int(L.ast_conv3x3_packed_numel(cout, cin)), device=w.device, dtype=torch.float32)
    check(L.ast_conv3x3_pack_weights_f32(ptr(w), ptr(out), cout, cin, stream_ptr(w.device)), "pack_conv3x3")
    return out


def pack_plan(n: int, w: int, pool: bool):
    """(G, gap) for side-by-side packing of n planes of width w (csrc/pack.hip): the group size
    that best fills the conv kernel's 32-pixel MFMA row tiles, if it gains >= 15%; (1, 0) else."""
    if os.environ.get("AST_CONV_PACK", "1") == "0" or n < 2 or w > 64 or (pool and w % 2):
        return 1, 0
    gap = 2 if pool else 1
    base = w / (-(-w // 32) * 32)
    best_u, best_g = base, 1
    for g in range(2, min(n, 8) + 1):
        wp = g * (w + gap) - gap
        u = n * w / (-(-n // g) * (-(-wp // 32) * 32))
        if u > best_u * 1.0001:
            best_u, best_g = u, g
    return (best_g, gap) if best_u >= 1.15 * base else (1, 0)


def conv3x3(x: torch.Tensor, w_packed: torch.Tensor, bias, cout: int, *, upsample: int = 1,
            pad_mode: str = "zeros", in_mean=None, in_std=None,
            want_pre: bool = False, want_act: bool = True, want_pool: bool = False, cfg: int = -1,
            x2: torch.Tensor | None = None, _pack: bool = True, _flops=None):
    """Fused [Upsample x2] -> pad(1) -> Conv3x3 -> (+bias) -> {pre, ReLU, ReLU+MaxPool2x2}.

    x2 (optional): a second batch with x's C, H, W; outputs hold x's images then x2's (one
    launch for a content batch and a style batch, no concatenation copy).
    Returns (pre, act, pool) with None for outputs not requested.
    """
    x = _dev(x, "x")
    if x.dim() != 4:
        raise HipOpError(f"x must be NCHW, got {tuple(x.shape)}")
    n1, cin, h_in, w_in = (int(s) for s in x.shape)
    n2 = 0
    if x2 is not None:
        x2 = _dev(x2, "x2")
        if x2.dim() != 4 or tuple(x2.shape[1:]) != tuple(x.shape[1:]) or x2.device != x.device:
            raise HipOpError(f"x2 {tuple(x2.shape)} must match x {tuple(x.shape)} in C, H, W")
        n2 = int(x2.shape[0])
    n = n1 + n2
    if w_packed.numel() != int(lib().ast_conv3x3_packed_numel(cout, cin)):
        raise HipOpError("packed weight does not match (cout, cin)")
    if bias is not None:
        bias = _dev(bias, "bias")
        if bias.numel() != cout:
            raise HipOpError("bias size mismatch")
    if (in_mean is None) != (in_std is None):
        raise HipOpError("in_mean and in_std go together")
    if in_mean is not None:
        in_mean, in_std = _dev(in_mean, "in_mean"), _dev(in_std, "in_std")
        if in_mean.numel() != cin or in_std.numel() != cin:
            raise HipOpError("normalisation stats must have cin entries")
    if pad_mode not in PAD_MODES:
        raise HipOpError(f"pad_mode must be one of {list(PAD_MODES)}")
    H, W = h_in * upsample, w_in * upsample
    mk = lambda hh, ww: torch.empty((n, cout, hh, ww), device=x.device, dtype=torch.float32)  # noqa: E731
    pre = mk(H, W) if want_pre else None
    act = mk(H, W) if want_act else None
    pool = mk(H // 2, W // 2) if want_pool else None
    if pool is not None and (H < 2 or W < 2):
        raise HipOpError("max-pool needs H, W >= 2")
    if pre is None and act is None and pool is None:
        raise HipOpError("conv3x3: no output requested")
    if cfg < 0:
        cfg = tuned_config(n, cin, h_in, w_in, cout, upsample, pad_mode, want_pool)
    G, gap = pack_plan(n, w_in, want_pool) if (_pack and pad_mode == "zeros" and upsample == 1
                                                and in_mean is None) else (1, 0)
    if G > 1:   # small planes: G images side by side per row band (identical results, fuller tiles)
        L = lib()
        ng, wp = -(-n // G), G * (w_in + gap) - gap
        xp = torch.empty((ng, cin, h_in, wp), device=x.device, dtype=torch.float32)
        check(L.ast_pack_images_f32(ptr(x), n1, ptr(x2), n2, cin, h_in, w_in, G, gap, ptr(xp),
                                    stream_ptr(x.device)), "pack")
        outs = conv3x3(xp, w_packed, bias, cout, want_pre=want_pre, want_act=want_act, want_pool=want_pool,
                       cfg=cfg, _pack=False, _flops=2 * n * H * W * cout * cin * 9)
        res = []
        for t, full, hh, ww in ((outs[0], pre, H, W), (outs[1], act, H, W), (outs[2], pool, H // 2, W // 2)):
            if t is not None:
                sp, wpp = (w_in + gap, wp) if hh == H else ((w_in + gap) // 2, wp // 2)
                check(L.ast_unpack_images_f32(ptr(t), n, cout, hh, ww, G, sp, wpp, ptr(full), stream_ptr(x.device)),
                      "unpack")
            res.append(full if t is not None else None)
        return tuple(res)
    flops = _flops if _flops is not None else 2 * n * H * W * cout * cin * 9
    tag = f"conv3x3 {cin}->{cout} {H}x{W} up{upsample} {pad_mode}"
    code = _timed(tag, flops, x.device, lambda: lib().ast_conv3x3_fwd_f32_cfg(
        cfg, ptr(x), ptr(x2), n2, ptr(w_packed), ptr(bias), ptr(pre), ptr(act), ptr(pool), ptr(in_mean),
        ptr(in_std), n1, cin, h_in, w_in, cout, upsample, PAD_MODES[pad_mode], stream_ptr(x.device)))
    check(code, "conv3x3")
    return pre, act, pool


# ------------------------------------------------------------------------------------------------
# Statistics / AdaIN
# ------------------------------------------------------------------------------------------------

def channel_stats(x: torch.Tensor, unbiased: bool = True, eps: float = 0.0):
    """Per-(n, c) mean and std over H, W, keepdim (model_util.py:3-8; calc_mean_std with eps)."""
    x = _dev(x, "x")
    if x.dim() != 4:
        raise HipOpError("channel_stats expects NCHW")
    n, c, h, w = x.shape
    mean = torch.empty((n, c, 1, 1), device=x.device, dtype=torch.float32)
    std = torch.empty_like(mean)
    check(lib().ast_channel_stats_f32(ptr(x), ptr(mean), ptr(std), n * c, h * w, 1 if unbiased else 0,
                                      float(eps), stream_ptr(x.device)), "channel_stats")
    return mean, std


def adain(content: torch.Tensor, style: torch.Tensor, alpha: float = 1.0, swap_style_stats: bool = True):
    """AdaIN (models.py:43-51) fused with the alpha blend of models.py:471."""
    if isinstance(content, torch.Tensor) and content.dtype == torch.bfloat16:
        return adain_bf16(content, style, alpha, swap_style_stats)
    content = _dev(content, "content_map")
    style = _dev(style, "style_map")
    if content.dim() != 4 or style.dim() != 4 or content.shape[:2] != style.shape[:2]:
        raise HipOpError(f"AdaIN needs NCHW maps with equal (N, C): {tuple(content.shape)} vs {tuple(style.shape)}")
    n, c, hc, wc = (int(s) for s in content.shape)
    hs, ws = int(style.shape[2]), int(style.shape[3])
    out = torch.empty_like(content)
    nbytes = 4 * (2 * content.numel() + style.numel())  # algorithmic: read c, read s, write out
    check(_timed(f"adain {c}ch {hc}x{wc}", -nbytes, content.device, lambda: lib().ast_adain_f32(
        ptr(content), ptr(style), ptr(out), n, c, hc, wc, hs, ws, float(alpha), 1 if swap_style_stats else 0,
        stream_ptr(content.device))), "adain")
    return out


def adain_stats(content: torch.Tensor, style_mean: torch.Tensor, style_std: torch.Tensor, alpha: float = 1.0,
                swap_style_stats: bool = True):
    """AdaIN of `content` [N, C, H, W] against given style statistics: [C] (one style shared by
    the batch) or [N, C] (any trailing 1-dims allowed), std unbiased as channel_stats."""
    content = _dev(content, "content_map")
    n, c, hc, wc = (int(s) for s in content.shape)
    m = _dev(style_mean, "style_mean").reshape(-1)
    s = _dev(style_std, "style_std").reshape(-1)
    if m.numel() != s.numel() or m.numel() not in (c, n * c):
        raise HipOpError(f"style statistics must have C={c} or N*C={n * c} entries, got {m.numel()}")
    out = torch.empty_like(content)
    check(lib().ast_adain_stats_f32(ptr(content), ptr(m), ptr(s), ptr(out), n, c, hc, wc,
                                    0 if m.numel() == c else c, float(alpha), 1 if swap_style_stats else 0,
                                    stream_ptr(content.device)), "adain_stats")
    return out


def _dev_typed(t: torch.Tensor, name: str, dtype: torch.dtype) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a tensor")
    if t.device.type != "cuda":
        raise HipOpError(f"{name} is on {t.device}; arbitrarystyletransfer_amd runs on MI355X (HIP) devices only")
    if t.dtype != dtype:
        raise HipOpError(f"{name} must be {dtype}, got {t.dtype}")
    return t.contiguous()


def adain_bf16(content: torch.Tensor, style: torch.Tensor, alpha: float = 1.0, swap_style_stats: bool = True):
    """AdaIN on bf16 maps (fp32 statistics and arithmetic, bf16 result)."""
    content = _dev_typed(content, "content_map", torch.bfloat16)
    style = _dev_typed(style, "style_map", torch.bfloat16)
    if content.dim() != 4 or style.dim() != 4 or content.shape[:2] != style.shape[:2]:
        raise HipOpError(f"AdaIN needs NCHW maps with equal (N, C): {tuple(content.shape)} vs {tuple(style.shape)}")
    n, c, hc, wc = (int(s) for s in content.shape)
    hs, ws = int(style.shape[2]), int(style.shape[3])
    out = torch.empty_like(content)
    nbytes = 2 * (2 * content.numel() + style.numel())
    check(_timed(f"adain bf16 {c}ch {hc}x{wc}", -nbytes, content.device, lambda: lib().ast_adain_bf16(
        ptr(content), ptr(style), ptr(out), n, c, hc, wc, hs, ws, float(alpha), 1 if swap_style_stats else 0,
        stream_ptr(content.device))), "adain_bf16")
    return out


def plane_normalize(x: torch.Tensor, mean: torch.Tensor, std: torch.Tensor):
    x = _dev(x, "x")
    mean, std = _dev(mean, "mean"), _dev(std, "std")
    n, c = x.shape[:2]
    hw = x.numel() // (n * c)
    out = torch.empty_like(x)
    check(lib().ast_plane_normalize_f32(ptr(x), ptr(mean), ptr(std), ptr(out), n * c, hw,
                                        stream_ptr(x.device)), "plane_normalize")
    return out


def mean_variance_norm(x: torch.Tensor):
    """models.py:64-68 (unbiased var + 1e-5)."""
    mean, std = channel_stats(x, unbiased=True, eps=1e-5)
    return plane_normalize(x, mean, std)


# ------------------------------------------------------------------------------------------------
# AdaAttN (models.py:70-115)
# ------------------------------------------------------------------------------------------------

ADAATTN_MAX_CHANNELS = 128


def adaattn(content: torch.Tensor, style: torch.Tensor, wq: torch.Tensor, wk: torch.Tensor, wv: torch.Tensor):
    """AdaAttN.forward (models.py:81-115) as HIP launches: instance-norm statistics, the Q/K/V 1x1
    projections, and one fused attention kernel (scores, online softmax, attention-weighted mean
    and std, `std * IN(content) + mean`); the Nq x Nk attention matrix is never materialised.
    content [N, C, H, W], style [N, C, Hs, Ws], both fp32 or both bf16 (bf16 storage, fp32
    accumulation); wq/wk/wv are the [C, C, 1, 1] (or [C, C]) Conv2d weights (any float dtype)."""
    if not isinstance(content, torch.Tensor) or not isinstance(style, torch.Tensor):
        raise TypeError("content_map and style_map must be tensors")
    if content.dtype == torch.bfloat16:
        dtype_code, content = 1, _dev_typed(content, "content_map", torch.bfloat16)
        style = _dev_typed(style, "style_map", torch.bfloat16)
    else:
        dtype_code, content, style = 0, _dev(content, "content_map"), _dev(style, "style_map")
    if content.dim() != 4 or style.dim() != 4 or content.shape[:2] != style.shape[:2]:
        raise HipOpError(f"AdaAttN needs NCHW maps with equal (N, C): {tuple(content.shape)} vs {tuple(style.shape)}")
    n, c, hc, wc = (int(s) for s in content.shape)
    hs, ws = int(style.shape[2]), int(style.shape[3])
    if hc * wc == 1 or hs * ws == 1:   # InstanceNorm2d's own error (models.py:78-80)
        raise ValueError("Expected more than 1 spatial element when training (InstanceNorm2d in AdaAttN)")
    if c > ADAATTN_MAX_CHANNELS:
        raise HipOpError(f"AdaAttN HIP kernel supports C <= {ADAATTN_MAX_CHANNELS}, got {c}")
    w = []
    for name, t in (("W_q", wq), ("W_k", wk), ("W_v", wv)):
        if t.device.type != "cuda":
            raise HipOpError(f"{name} is on {t.device}; arbitrarystyletransfer_amd runs on MI355X (HIP) devices only")
        t = t.detach().to(torch.float32).contiguous()
        if t.numel() != c * c:
            raise HipOpError(f"{name} must be [{c}, {c}, 1, 1], got {tuple(t.shape)}")
        w.append(t)
    out = torch.empty_like(content)
    nbytes = lib().ast_adaattn_workspace_bytes(dtype_code, n, c, hc, wc, hs, ws)
    ws_buf = torch.empty((nbytes,), dtype=torch.uint8, device=content.device)
    flops = 6 * n * c * (hc * wc) * (hs * ws)   # S (2C) + P[V, V^2] (4C) per score
    tag = f"adaattn{' bf16' if dtype_code else ''} {c}ch {hc}x{wc}<-{hs}x{ws}"
    check(_timed(tag, flops, content.device, lambda: lib().ast_adaattn_fwd(
        dtype_code, ptr(content), ptr(style), ptr(w[0]), ptr(w[1]), ptr(w[2]), ptr(out), ptr(ws_buf), nbytes,
        n, c, hc, wc, hs, ws, stream_ptr(content.device))), "adaattn")
    return out


def emd_rows(hx: torch.Tensor, hy: torch.Tensor):
    """EarthMoversDistanceLoss.forward (losses.py:11-22) on [B, 256] histograms: [B] values."""
    hx, hy = _dev(hx, "x"), _dev(hy, "y")
    if hx.dim() != 2 or hx.shape != hy.shape or hx.shape[1] != 256:
        raise HipOpError(f"earth movers: expected two [B, 256] tensors, got {tuple(hx.shape)} / {tuple(hy.shape)}")
    b = hx.shape[0]
    acc_n = int(lib().ast_loss_acc_floats())
    accs = torch.zeros((b, acc_n), device=hx.device, dtype=torch.float32)   # one loss accumulator per row
    for i in range(b):   # one scalar per row: the kernel accumulates weight/n * row sums
        check(lib().ast_emd_loss_f32(ptr(hx[i:i + 1]), ptr(hy[i:i + 1]), 1, 1.0, None, ptr(accs[i]), None,
                                     stream_ptr(hx.device)), "emd")
    return accs[:, 0]
