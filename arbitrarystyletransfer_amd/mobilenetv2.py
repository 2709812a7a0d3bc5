"""The reference's MobileNet-style blocks (mobilenetv2.py) on HIP kernels.

Same class names, constructor signatures and module trees as the reference, so state dicts load
unchanged; the forwards run on the fused kernels of csrc/mobilenet.hip (C ABI `ast_mb_*`):

    DepthWiseConv  (mobilenetv2.py:95-181)  ast_mb_expand_dw -> ast_mb_se_fold -> ast_mb_pw
    conv_3x3_bn    (mobilenetv2.py:38-43)   ast_mb_conv3x3_dense
    SELayer        (mobilenetv2.py:63-81)   fused into DepthWiseConv (pool sums + gate folding)

Eval mode (the inference path): BatchNorm runs with its running statistics and
is folded into the conv weights. Training mode or autograd recording (train_autoencoder.py,
train.py's ASTTrainer) dispatches to the composable training kernels of mbtrain.py
(csrc/mbtrain.hip: batch statistics, running-stat updates, every intermediate kept for backward).
Activations are stored in the parameters' dtype (float32, or bfloat16 after
`.to(torch.bfloat16)`); arithmetic and accumulation are fp32.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn

from . import mbtrain, ops
from ._lib import HipOpError, check, lib, ptr, stream_ptr, workspace

__all__ = ["_make_divisible", "conv_3x3_bn", "SELayer", "DepthWiseConv"]

DTYPE_CODE = {torch.float32: 0, torch.bfloat16: 1}

# When a list, every block forward appends its block-fused minimum HBM bytes (read the block input
# once, write its output once) — bench.py's config-5 roofline denominator.
IO_TRACE = None
DW_TRACE = None   # bench.py: per expand_dw launch, the depthwise multiply-adds (VALU work)
# The fused block pair (ast_mb_expand_dw_pw: no hidden-width tensor in memory) for the shapes it
# supports, bit-identical to expand_dw + se_fold + pw; on by default since round 4 (its outputs leave
# as 8-byte pieces: DESIGN.md §3, "Fused block pair"). AST_MB_EDPW=0 selects the unfused chain.
FUSED_PAIR = os.environ.get("AST_MB_EDPW", "1") == "1"


def _trace_io(nbytes: int) -> None:
    if IO_TRACE is not None:
        IO_TRACE.append(nbytes)


def _make_divisible(v, divisor, min_value=None):
    """mobilenetv2.py:18-35: round v to a multiple of divisor, never below 90% of v."""
    if min_value is None:
        min_value = divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


def _round_up(a: int, b: int) -> int:
    return (a + b - 1) // b * b


def act_dtype(module: nn.Module) -> torch.dtype:
    dt = next(module.parameters()).dtype
    if dt not in DTYPE_CODE:
        raise HipOpError(f"MobileNet blocks run in float32 or bfloat16, not {dt}")
    return dt


def check_inference(x: torch.Tensor, module: nn.Module) -> None:
    if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in module.parameters())):
        raise NotImplementedError("the fused MobileNet-variant kernels fold eval-mode BatchNorm and keep no "
                                  "intermediates for autograd; this module has eval-mode BatchNorm under autograd: "
                                  "run it under torch.no_grad(), or in train mode (mbtrain.py training kernels)")


_ED_WS = {}


def _expand_dw(dt, x1, x2, c1, n, cin, h, w, up, w1p, b1, hid, cin_pad, wd, bd, k, s, d, pool, ho, wo, st):
    """ast_mb_expand_dw with its workspace (the per-tile SE-pool sums, reduced in tile order)."""
    key = (DTYPE_CODE[dt], x2 is not None, c1, n, cin, h, w, up, w1p is not None, hid, cin_pad, k, s, ho, wo)
    nws = _ED_WS.get(key)
    if nws is None:
        nws = _ED_WS[key] = int(lib().ast_mb_expand_dw_workspace_floats(*(int(v) for v in key)))
    ws = workspace(nws, pool.device)
    return lib().ast_mb_expand_dw(DTYPE_CODE[dt], ptr(x1), ptr(x2), c1, n, cin, h, w, up, ptr(w1p), ptr(b1), hid,
                                  cin_pad, ptr(wd), ptr(bd), k, s, ptr(d), ptr(pool), ho, wo, ptr(ws), ws.numel(), st)


def _act_input(x: torch.Tensor, dt: torch.dtype, name: str = "x") -> torch.Tensor:
    if not isinstance(x, torch.Tensor):
        raise TypeError(f"{name} must be a tensor")
    if x.device.type != "cuda":
        raise HipOpError(f"{name} is on {x.device}; arbitrarystyletransfer_amd runs on MI355X (HIP) devices only")
    if x.dim() != 4:
        raise HipOpError(f"{name} must be NCHW, got shape {tuple(x.shape)}")
    if x.dtype != dt:
        raise HipOpError(f"{name} is {x.dtype} but the block's parameters are {dt}")
    return x.contiguous()


def _stamp(module: nn.Module, dt, device):
    ts = list(module.parameters()) + list(module.buffers())
    return (dt, device) + tuple((t.data_ptr(), t._version, ops.weight_epoch(t)) for t in ts)


class _Conv3x3HS(nn.Sequential):
    """conv_3x3_bn (mobilenetv2.py:38-43): Conv2d(3->16, 3x3, reflect pad 1, no bias) + Hardswish,
    one VALU launch. The image may be float32 or bfloat16; the output has the parameters' dtype."""

    def forward(self, x):
        conv = self[0]
        if mbtrain.wants_training_path(self, x):
            from . import functional as Fn
            y = Fn.DecoderConvFn.apply(x.float().contiguous(), conv.weight, None,
                                       ops.pack_conv3x3(conv.weight.detach().float()), 1, False)
            return mbtrain.HardswishFn.apply(y)
        check_inference(x, self)
        dt = act_dtype(self)
        if not isinstance(x, torch.Tensor) or x.device.type != "cuda" or x.dim() != 4:
            raise HipOpError("conv_3x3_bn expects an NCHW tensor on a HIP device")
        if x.shape[1] != conv.in_channels:
            raise HipOpError(f"expected {conv.in_channels} input channels, got {x.shape[1]}")
        x = (x if x.dtype == dt == torch.bfloat16 else x.float()).contiguous()
        n, _, h, w = x.shape
        stamp = _stamp(self, dt, x.device)
        if getattr(self, "_cache_stamp", None) != stamp:
            self._w = conv.weight.detach().float().contiguous()
            self._cache_stamp = stamp
        y = torch.empty((n, conv.out_channels, h, w), device=x.device, dtype=dt)
        nbytes = x.numel() * x.element_size() + y.numel() * y.element_size()
        _trace_io(nbytes)
        check(ops._timed("mb dense3x3", -nbytes, x.device, lambda: lib().ast_mb_conv3x3_dense(
            DTYPE_CODE[x.dtype], DTYPE_CODE[dt], ptr(x), ptr(self._w), None, ptr(y), n, conv.in_channels, conv.out_channels, h, w, 1,
            stream_ptr(x.device))), "conv_3x3_bn")
        return y


def conv_3x3_bn(inp, oup, stride):
    """mobilenetv2.py:38-43 (the BatchNorm is commented out there, so none here either)."""
    if stride != 1:
        raise NotImplementedError("conv_3x3_bn: only stride 1 is used by the reference Encoder (conf.py:77)")
    return _Conv3x3HS(nn.Conv2d(inp, oup, 3, stride, 1, bias=False, padding_mode="reflect"), nn.Hardswish(True))


class SELayer(nn.Module):
    """mobilenetv2.py:63-81 (same parameters). Its forward is fused into DepthWiseConv: the dw
    kernel accumulates the AdaptiveAvgPool sums and ast_mb_se_fold evaluates the MLP and folds the
    Hardtanh(0,1) gate into the following 1x1 conv."""

    def __init__(self, channel, reduction=4):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        mid = _make_divisible(channel // reduction, 8)
        self.fc = nn.Sequential(nn.Linear(channel, mid), nn.ReLU(inplace=True), nn.Linear(mid, channel),
                                nn.Hardtanh(0.0, 1.0))

    def forward(self, x):
        raise NotImplementedError("SELayer runs fused inside DepthWiseConv on the HIP path")


class _BlockPlan:
    __slots__ = ("w1p", "b1", "cin_pad", "wd", "bd", "fc1w", "fc1b", "fc2w", "fc2b", "red", "w2", "b2",
                 "hid_pad", "cout_pad")


class DepthWiseConv(nn.Module):
    """mobilenetv2.py:95-181 (inverted residual with SE), same `_layers` layout.

    forward(x) == the reference forward with BatchNorm in eval mode. `forward(x, x2)` consumes
    torch.cat((x, x2), 1) without materialising it (AutoEncoder/AST ada_out, models.py:335,565)."""

    def __init__(self, inp, oup, stride, expand_ratio, kernel_size=3, use_norm=False, padding=0,
                 use_identity=True, use_relu=False):
        super().__init__()
        hidden_dim = round(inp * expand_ratio)
        self.identity = stride == 1 and inp == oup and use_identity
        self.inp, self.oup, self.stride, self.kernel_size = inp, oup, stride, kernel_size
        self.expand_ratio, self.use_norm, self.hidden_dim = expand_ratio, use_norm, hidden_dim
        layers = []
        if expand_ratio == 1:
            layers.append(nn.ReflectionPad2d((1, 1, 1, 1)))
            layers.append(nn.Conv2d(hidden_dim, hidden_dim, kernel_size, stride, 0, groups=hidden_dim, bias=False))
            if use_norm:
                layers.append(nn.BatchNorm2d(hidden_dim, affine=True, track_running_stats=True))
            layers.append(nn.Hardswish(True))
            layers.append(SELayer(hidden_dim))
            layers.append(nn.Conv2d(hidden_dim, oup, 1, 1, 0, bias=False))
            if use_norm:
                layers.append(nn.BatchNorm2d(oup, affine=True, track_running_stats=True))
        else:
            layers.append(nn.Conv2d(inp, hidden_dim, 1, 1, 0, bias=False))
            if use_norm:
                layers.append(nn.BatchNorm2d(hidden_dim, affine=True, track_running_stats=True))
            layers.append(nn.Hardswish(True))
            layers.append(nn.Conv2d(hidden_dim, hidden_dim, kernel_size, stride, (kernel_size - 1) // 2,
                                    groups=hidden_dim, bias=False, padding_mode="reflect"))
            if use_norm:
                layers.append(nn.BatchNorm2d(hidden_dim, affine=True, track_running_stats=True))
            layers.append(nn.Hardswish(True))
            layers.append(SELayer(hidden_dim))
            layers.append(nn.Conv2d(hidden_dim, oup, 1, 1, 0, bias=False))
            if use_norm:
                layers.append(nn.BatchNorm2d(oup, affine=True, track_running_stats=True))
        self._layers = nn.ModuleList(layers)
        self._initialize_weights()

    def _initialize_weights(self):
        """mobilenetv2.py:167-181."""
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                n = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / n))
                if m.bias is not None:
                    m.bias.data.zero_()
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
            elif isinstance(m, nn.Linear):
                m.weight.data.normal_(0, 0.01)
                m.bias.data.zero_()

    # -- folded, packed parameters -------------------------------------------------------------
    def _fold(self, i):
        """Weight of conv _layers[i] with a following eval BatchNorm folded in: (w, b or None)."""
        conv = self._layers[i]
        w = conv.weight.detach().float()
        bn = self._layers[i + 1] if i + 1 < len(self._layers) else None
        if not isinstance(bn, nn.BatchNorm2d):
            return w, None
        s = bn.weight.detach().float() / torch.sqrt(bn.running_var.detach().float() + bn.eps)
        return w * s.view(-1, 1, 1, 1), bn.bias.detach().float() - bn.running_mean.detach().float() * s

    def _fold_into(self, i, rows, ld, want_bias):
        """_fold of conv _layers[i] as one HIP launch (ast_mb_fold_bn_f32: the same roundings),
        into a zero-padded [rows][ld] fp32 buffer; the bias (zeros without a BatchNorm) or None."""
        conv = self._layers[i]
        bn = self._layers[i + 1] if i + 1 < len(self._layers) else None
        has_bn = isinstance(bn, nn.BatchNorm2d)
        w = conv.weight.detach()
        if w.dtype != torch.float32 or not w.is_contiguous():
            w = w.float().contiguous()
        cout, k = int(w.shape[0]), int(w[0].numel())
        out = torch.empty((rows, ld), device=w.device, dtype=torch.float32)
        b = torch.empty(cout, device=w.device, dtype=torch.float32) if (want_bias or has_bn) else None
        args = [None] * 4
        if has_bn:
            args = [t.detach() if t.dtype == torch.float32 else t.detach().float()
                    for t in (bn.weight, bn.bias, bn.running_mean, bn.running_var)]
            args = [t if t.is_contiguous() else t.contiguous() for t in args]
        check(lib().ast_mb_fold_bn_f32(ptr(w), cout, k, *(ptr(t) for t in args), float(bn.eps) if has_bn else 0.0,
                                       int(has_bn), ptr(out), ld, rows, ptr(b), stream_ptr(w.device)),
              "fold BatchNorm")
        return out, b

    def _plan(self, dt, device) -> _BlockPlan:
        stamp = _stamp(self, dt, device)
        if getattr(self, "_plan_stamp", None) == stamp:
            return self._pl
        convs = [i for i, m in enumerate(self._layers) if isinstance(m, nn.Conv2d)]
        se = next(m for m in self._layers if isinstance(m, SELayer))
        p = _BlockPlan()
        hid, cout = self.hidden_dim, self.oup
        if self.expand_ratio == 1:
            i_dw, i_pw = convs
            p.w1p = p.b1 = None
            p.cin_pad = 0
        else:
            i_pw1, i_dw, i_pw = convs
            p.cin_pad = _round_up(self.inp, 16 if dt == torch.bfloat16 else 4)
            w1p, p.b1 = self._fold_into(i_pw1, _round_up(hid, 16), p.cin_pad, True)
            p.w1p = w1p if dt == torch.float32 else w1p.to(dt).contiguous()
        k2 = self._layers[i_dw].weight[0].numel()
        p.wd, p.bd = self._fold_into(i_dw, hid, k2, True)
        fc1, fc2 = se.fc[0], se.fc[2]
        p.fc1w = fc1.weight.detach().float().contiguous()
        p.fc1b = fc1.bias.detach().float().contiguous()
        p.fc2w = fc2.weight.detach().float().contiguous()
        p.fc2b = fc2.bias.detach().float().contiguous()
        p.red = fc1.out_features
        p.w2, p.b2 = self._fold_into(i_pw, cout, hid, False)
        p.hid_pad = _round_up(hid, 32)
        p.cout_pad = _round_up(cout, 16)
        self._pl, self._plan_stamp = p, stamp
        return p

    def _fused_ok(self, dt, cin, cin_pad, hid, cout, k, s, ho, wo):
        """The fused block pair (ast_mb_expand_dw_pw) runs this block shape."""
        return bool(lib().ast_mb_expand_dw_pw_supported(DTYPE_CODE[dt], 0, cin, cin_pad, hid, cout, k, s, 1, ho, wo))

    # -- forward --------------------------------------------------------------------------------
    def forward(self, x, x2=None):
        return self.run(x, x2, 1)

    def run(self, x, x2=None, up: int = 1):
        """Block forward on x (or cat(x, x2) along channels), after a nearest x`up` upsample."""
        if mbtrain.wants_training_path(self, x, x2) or (self.use_norm and self.training):
            return mbtrain.block_forward(self, x, x2, up)   # layer by layer, with backward
        if self.use_norm and self.training:
            raise NotImplementedError("DepthWiseConv with BatchNorm in training mode (batch statistics) is not "
                                      "implemented on the HIP path; call .eval() (running statistics)")
        check_inference(x, self)
        dt = act_dtype(self)
        x = _act_input(x, dt)
        n, c1, h, w = (int(s) for s in x.shape)
        cin = c1
        if x2 is not None:
            x2 = _act_input(x2, dt, "x2")
            if x2.shape[0] != n or x2.shape[2:] != x.shape[2:]:
                raise HipOpError("x and x2 must agree in N, H, W")
            cin += int(x2.shape[1])
            if self.identity:
                raise HipOpError("a residual block cannot take a split input")
        if cin != self.inp:
            raise HipOpError(f"expected {self.inp} input channels, got {cin}")
        k, s = self.kernel_size, self.stride
        pad = (k - 1) // 2
        if self.expand_ratio == 1 and (k != 3 or s != 1):
            raise NotImplementedError("ratio-1 DepthWiseConv is implemented for kernel 3, stride 1 (models.py:262)")
        hd, wd = h * up, w * up
        if hd <= pad or wd <= pad:
            raise HipOpError(f"reflection padding {pad} needs a larger input than {hd}x{wd}")
        ho, wo = (hd + 2 * pad - k) // s + 1, (wd + 2 * pad - k) // s + 1
        p = self._plan(dt, x.device)
        hid, cout = self.hidden_dim, self.oup
        dev, st = x.device, stream_ptr(x.device)
        es = x.element_size()
        fused = (FUSED_PAIR and x2 is None and up == 1 and p.w1p is not None
                 and self._fused_ok(dt, cin, p.cin_pad, hid, cout, k, s, ho, wo))
        d = None if fused else torch.empty((n, hid, ho, wo), device=dev, dtype=dt)
        pool = torch.empty((n, hid), device=dev, dtype=torch.float32)
        nb1 = es * (n * cin * h * w + (d.numel() if d is not None else 0))
        tag = f"mb expand_dw k{k}s{s}{' up' if up == 2 else ''} {cin}->{hid} {ho}x{wo}"
        if (dt == torch.bfloat16 and p.w1p is not None and p.cin_pad >= 256 and p.cin_pad % 32 == 0
                and hid % 128 == 0 and s == 1 and up == 1 and k == 3):
            # too wide for the fused kernels' LDS/registers (ada_out, 256 -> 768): the expand as a GEMM
            # with Hardswish into a bf16 hidden tensor, then the ratio-1 depthwise pass on it
            hmid = torch.empty((n, hid, h, w), device=dev, dtype=dt)
            check(ops._timed(tag + " gemm", -es * (n * cin * h * w + hmid.numel()), dev,
                             lambda: lib().ast_mb_expand_gemm(
                                 DTYPE_CODE[dt], ptr(x), ptr(x2), c1, n, cin, h, w, ptr(p.w1p), ptr(p.b1), hid,
                                 p.cin_pad, ptr(hmid), st)), "DepthWiseConv expand GEMM")
            check(ops._timed(tag + " dw", -es * (hmid.numel() + d.numel()), dev,
                             lambda: _expand_dw(dt, hmid, None, hid, n, hid, h, w, 1, None, None, hid, 0, p.wd, p.bd,
                                                k, s, d, pool, ho, wo, st)),
                  "DepthWiseConv dw")
        elif fused:
            # the fused pair: pool-only pass (no D), SE fold, then expand + depthwise recomputed with
            # the gated pw-linear conv applied in the kernel (csrc/mb_ed4.hip expand_dw_pw4_kernel)
            check(ops._timed(f"mb expand_dw k{k}s{s} pool {cin}->{hid} {ho}x{wo}", -es * n * cin * h * w, dev,
                             lambda: _expand_dw(dt, x, None, c1, n, cin, h, w, 1, p.w1p, p.b1, hid, p.cin_pad, p.wd,
                                                p.bd, k, s, None, pool, ho, wo, st)),
                  "DepthWiseConv pool pass")
        else:
            check(ops._timed(tag, -nb1, dev,
                             lambda: _expand_dw(dt, x, x2, c1, n, cin, h, w, up, p.w1p, p.b1, hid, p.cin_pad, p.wd,
                                                p.bd, k, s, d, pool, ho, wo, st)),
                  "DepthWiseConv expand+dw")
        wg = torch.empty((n, p.cout_pad, p.hid_pad), device=dev, dtype=dt)
        check(lib().ast_mb_se_fold(DTYPE_CODE[dt], ptr(pool), n, hid, ho * wo, ptr(p.fc1w), ptr(p.fc1b), p.red,
                                   ptr(p.fc2w), ptr(p.fc2b), ptr(p.w2), cout, p.cout_pad, p.hid_pad, ptr(wg), st),
              "DepthWiseConv SE")
        out = torch.empty((n, cout, ho, wo), device=dev, dtype=dt)
        _trace_io(es * (n * cin * h * w + out.numel()))
        if DW_TRACE is not None:   # depthwise FMAs of the expand_dw launch (bench.py's VALU figure)
            DW_TRACE.append(n * hid * ho * wo * k * k)
        res = x if self.identity else None
        if fused:
            nb3 = es * (n * cin * h * w + out.numel() + (res.numel() if res is not None else 0))
            check(ops._timed(f"mb expand_dw_pw k{k}s{s} {cin}->{hid}->{cout} {ho}x{wo}", -nb3, dev,
                             lambda: lib().ast_mb_expand_dw_pw(
                                 DTYPE_CODE[dt], ptr(x), n, cin, h, w, ptr(p.w1p), ptr(p.b1), hid, p.cin_pad,
                                 ptr(p.wd), ptr(p.bd), k, ptr(wg), cout, p.cout_pad, p.hid_pad, ptr(p.b2), ptr(res),
                                 ptr(out), st)), "DepthWiseConv fused expand+dw+pw")
            return out
        nb2 = es * (d.numel() + out.numel() + (res.numel() if res is not None else 0))
        check(ops._timed(f"mb pw {hid}->{cout} {ho}x{wo}", -nb2, dev, lambda: lib().ast_mb_pw(
            DTYPE_CODE[dt], ptr(d), n, hid, p.hid_pad, ho, wo, ptr(wg), p.cout_pad * p.hid_pad, ptr(p.b2), cout,
            p.cout_pad, ptr(res), 1 if (res is not None and up == 2) else 0, ptr(out), st)), "DepthWiseConv pw")
        return out
