"""torch.ops.ast_hip.*: the hot-path ops as PyTorch custom operators -- the path the drop-in
modules (models.py, mobilenetv2.py) and losses.py call ("What the C++ side
exports").

Every op launches the same C-ABI kernels of libast_hip.so as the ctypes helpers in ops.py /
functional.py (its implementation IS those helpers), on PyTorch's current HIP stream. Each op has
a fake (meta) implementation, so torch.compile / FakeTensor tracing sees shapes without running
kernels -- `torch.compile(models.AdaINStyleTransfer(), fullgraph=True)` traces the forward with no
graph break -- and the differentiable ones carry their backward formula
(torch.library.register_autograd), whose kernels are the HIP backward kernels (conv dgrad / wgrad,
AdaIN backward, the fused loss gradients). The native C++ registration (csrc/torch_ops.cpp,
libast_torch_ops.so: adain, channel_stats, conv3x3_pack, conv3x3_fwd, gram) shares the namespace;
gram gets its autograd formula here.

Op                      reference (file:line)                       autograd
conv3x3                 models.py:199-240 (encoder), :598-628 (decoder)   dx, dW, db
adain_map               models.py:43-51 (+ alpha blend :471)         d content, d style (fp32)
gram (C++)              losses.py:105-109                            d feat
content_mvn_loss        losses.py:124-126 on mean_variance_norm      d x
style_loss              losses.py:128-139                            d x
huber_loss              losses.py:124-126 (compute_content_loss)     d x, d y
tv_loss                 losses.py:90-103                             d img
hist_loss               losses.py:84-87 (SingleDimHist + EMD)        d x
range_loss              train.py:259                                 d x
sqdiff_mean             train.py:268                                 d x
mb_expand_dw            mobilenetv2.py:153-161 (to the SE pool)      -- (eval BN folded: inference)
mb_se_fold              mobilenetv2.py:63-81 folded into the pw conv --
mb_pw                   mobilenetv2.py:162-165                       --
mb_expand_gemm          models.py:335 (ada_out expand half)          --
mb_conv3x3_dense        mobilenetv2.py:38-43, models.py:300-316      --
The MobileNet inference ops fold eval-mode BatchNorm; training runs the composable kernels of
mbtrain.py (their own autograd), as the drop-in DepthWiseConv does.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
from torch import Tensor
from torch.library import custom_op, register_autograd, register_fake

from . import functional as Fn
from . import ops, torch_ops
from ._lib import check, lib, loss_accumulator, ptr, stream_ptr, workspace

torch_ops.load()   # the native registrations (and libast_hip.so) first: no fallback

PADS = ("zeros", "reflect")


def _empty(like: Tensor) -> Tensor:
    return like.new_empty((0,))


# ------------------------------------------------------------------------------------------------
# conv3x3: [Upsample x2] -> pad(1) -> Conv3x3 -> (+bias) -> {pre, ReLU, ReLU + MaxPool2x2}
# ------------------------------------------------------------------------------------------------

@custom_op("ast_hip::conv3x3", mutates_args=())
def conv3x3(x: Tensor, weight: Tensor, w_packed: Tensor, bias: Optional[Tensor], upsample: int, pad_mode: int,
            in_mean: Optional[Tensor], in_std: Optional[Tensor], want_pre: bool, want_act: bool, want_pool: bool,
            x2: Optional[Tensor]) -> Tuple[Tensor, Tensor, Tensor]:
    """Outputs (pre, act, pool); unrequested ones are empty. `weight` [cout, cin, 3, 3] is the
    unpacked filter (the backward's dW and transposed pack come from it); `w_packed` its pack."""
    pre, act, pool = ops.conv3x3(x, w_packed, bias, int(weight.shape[0]), upsample=upsample,
                                 pad_mode=PADS[pad_mode], in_mean=in_mean, in_std=in_std, want_pre=want_pre,
                                 want_act=want_act, want_pool=want_pool, x2=x2)
    return (pre if pre is not None else _empty(x), act if act is not None else _empty(x),
            pool if pool is not None else _empty(x))


@register_fake("ast_hip::conv3x3")
def _(x, weight, w_packed, bias, upsample, pad_mode, in_mean, in_std, want_pre, want_act, want_pool, x2):
    n = x.shape[0] + (x2.shape[0] if x2 is not None else 0)
    cout, H, W = weight.shape[0], x.shape[2] * upsample, x.shape[3] * upsample
    mk = lambda want, h, w: x.new_empty((n, cout, h, w)) if want else x.new_empty((0,))  # noqa: E731
    return mk(want_pre, H, W), mk(want_act, H, W), mk(want_pool, H // 2, W // 2)


def _conv_setup(ctx, inputs, output):
    x, weight, w_packed, bias, upsample, pad_mode, in_mean, in_std, want_pre, want_act, want_pool, x2 = inputs
    if x2 is not None:
        raise NotImplementedError("ast_hip::conv3x3: the two-batch form (x2) has no backward; call it per batch")
    pre, act, _ = output
    if pad_mode == 0 and not want_pre:
        raise NotImplementedError("ast_hip::conv3x3 (zero padding) under autograd needs want_pre=True "
                                  "(the ReLU / max-pool backward reads the pre-activation)")
    if pad_mode == 1 and want_pool:
        raise NotImplementedError("ast_hip::conv3x3 (reflect padding) under autograd: no max-pool backward")
    mask = pre if pad_mode == 0 else (act if want_act else None)
    ctx.save_for_backward(x, weight, mask, in_mean, in_std)
    ctx.cfg = (upsample, pad_mode, bias is not None, want_act)


def _conv_backward(ctx, g_pre, g_act, g_pool):
    x, weight, mask, mean, std = ctx.saved_tensors
    upsample, pad_mode, has_bias, want_act = ctx.cfg
    cout = int(weight.shape[0])
    n, cin, hin, win = x.shape
    H, W = hin * upsample, win * upsample
    nz = lambda t: t if (t is not None and t.numel()) else None  # noqa: E731
    dx = dw = db = None
    if pad_mode == 0:   # the encoder walk (EncoderConvFn): act backward, dgrad, wgrad
        gp, ga, gq = nz(g_pre), nz(g_act), nz(g_pool)
        dy = torch.empty_like(mask)
        check(lib().ast_conv_act_backward_f32(ptr(mask), ptr(gp.contiguous() if gp is not None else None),
                                              ptr(ga.contiguous() if ga is not None else None),
                                              ptr(gq.contiguous() if gq is not None else None), ptr(dy),
                                              n * cout, H, W, stream_ptr(x.device)), "conv_act_backward")
        if ctx.needs_input_grad[0]:
            dx = Fn.conv_input_grad_same(dy, weight, std.view(-1) if std is not None else None)
        if ctx.needs_input_grad[1] or (has_bias and ctx.needs_input_grad[3]):
            xin = Fn.normalize_image(x, mean, std) if mean is not None else x
            dw, db = Fn.conv_weight_grad(xin, dy, cout, with_bias=has_bias)
    else:               # the decoder walk (DecoderConvFn.backward): ReLU mask, input grad + border fold, wgrad
        g = nz(g_act) if want_act else nz(g_pre)
        g = g.contiguous()
        if want_act:
            dy = torch.empty_like(g)
            check(lib().ast_relu_mask_f32(ptr(g), ptr(mask), ptr(dy), g.numel(), stream_ptr(g.device)), "relu_mask")
        else:
            dy = g
        if ctx.needs_input_grad[0]:
            dx = Fn.conv_input_grad(dy, weight, upsample, "reflect")
        if ctx.needs_input_grad[1] or (has_bias and ctx.needs_input_grad[3]):
            dw, db = Fn.conv_weight_grad(x, dy, cout, upsample, "reflect", has_bias)
    return dx, dw, None, db, None, None, None, None, None, None, None, None


register_autograd("ast_hip::conv3x3", _conv_backward, setup_context=_conv_setup)


# ------------------------------------------------------------------------------------------------
# AdaIN (+ alpha blend)
# ------------------------------------------------------------------------------------------------

@custom_op("ast_hip::adain_map", mutates_args=())
def adain_map(content: Tensor, style: Tensor, alpha: float, swap_style_stats: bool) -> Tensor:
    return ops.adain(content, style, alpha=alpha, swap_style_stats=swap_style_stats)


@register_fake("ast_hip::adain_map")
def _(content, style, alpha, swap_style_stats):
    return torch.empty_like(content)


def _adain_setup(ctx, inputs, output):
    content, style, alpha, swap = inputs
    if content.dtype != torch.float32:
        raise NotImplementedError("ast_hip::adain_map backward runs in float32")
    ctx.save_for_backward(content, style)
    ctx.alpha, ctx.swap = alpha, swap


def _adain_backward(ctx, g):
    content, style = ctx.saved_tensors
    n, c, hc, wc = content.shape
    hs, ws = style.shape[2:]
    dc = torch.empty_like(content) if ctx.needs_input_grad[0] else None
    ds = torch.empty_like(style) if ctx.needs_input_grad[1] else None
    if dc is not None or ds is not None:
        check(lib().ast_adain_backward_f32(ptr(content), ptr(style), ptr(g.contiguous()), ptr(dc), ptr(ds), n, c, hc,
                                           wc, hs, ws, float(ctx.alpha), 1 if ctx.swap else 0,
                                           stream_ptr(content.device)), "adain_backward")
    return dc, ds, None, None


register_autograd("ast_hip::adain_map", _adain_backward, setup_context=_adain_setup)


# ------------------------------------------------------------------------------------------------
# gram (native registration) + its backward
# ------------------------------------------------------------------------------------------------

def _gram_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[0])


def _gram_backward(ctx, dg):
    (f,) = ctx.saved_tensors
    b, c, h, w = f.shape
    df = torch.empty_like(f)
    check(lib().ast_gram_backward_f32(ptr(f), ptr(dg.contiguous()), ptr(df), None, None, b, c, h * w,
                                      1.0 / (c * h * w), None, 0, stream_ptr(f.device)), "gram_backward")
    return df


register_autograd("ast_hip::gram", _gram_backward, setup_context=_gram_setup)


# ------------------------------------------------------------------------------------------------
# Losses: value ops with the gradient state as extra (non-differentiable) outputs
# ------------------------------------------------------------------------------------------------

def _acc(like):
    return loss_accumulator(like.device, pooled=False)   # custom-op outputs: storage of their own


@custom_op("ast_hip::content_mvn_loss", mutates_args=())
def content_mvn_loss(x: Tensor, y: Tensor, weight: float, want_grad: bool) -> Tuple[Tensor, Tensor]:
    """weight * compute_content_loss(mean_variance_norm(x), mean_variance_norm(y)); second output:
    the per-plane statistics of the backward (empty unless want_grad)."""
    n, c = x.shape[:2]
    acc = _acc(x)
    pstats = torch.empty((n * c, 6), device=x.device) if want_grad else _empty(x)
    Fn.mvn_huber(x, y, weight, acc, pstats if want_grad else None)
    return acc[0], pstats


@register_fake("ast_hip::content_mvn_loss")
def _(x, y, weight, want_grad):
    return x.new_empty(()), x.new_empty((x.shape[0] * x.shape[1], 6) if want_grad else (0,))


def _mvn_setup(ctx, inputs, output):
    x, y, weight, want_grad = inputs
    if not want_grad:
        raise NotImplementedError("ast_hip::content_mvn_loss under autograd needs want_grad=True")
    ctx.save_for_backward(x, y, output[1])
    ctx.weight = weight


def _mvn_backward(ctx, g, _):
    x, y, pstats = ctx.saved_tensors
    n, c = x.shape[:2]
    dx = torch.empty_like(x)
    check(lib().ast_mvn_huber_backward_f32(ptr(x), ptr(y), ptr(pstats), n * c, x[0, 0].numel(), ctx.weight,
                                           ptr(g.contiguous()), ptr(dx), 0, stream_ptr(x.device)), "mvn_huber_backward")
    return dx, None, None, None


register_autograd("ast_hip::content_mvn_loss", _mvn_backward, setup_context=_mvn_setup)


@custom_op("ast_hip::style_loss", mutates_args=())
def style_loss(x: Tensor, y: Tensor, weight: float, want_grad: bool) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """weight * compute_style_loss(x, y); extra outputs: dG, row_a, row_b of the gradient."""
    acc = _acc(x)
    dg, ra, rb = Fn._style_terms(x, y, weight, acc, want_grad=want_grad)
    e = lambda: _empty(x)  # noqa: E731
    return acc[0], dg if dg is not None else e(), ra if ra is not None else e(), rb if rb is not None else e()


@register_fake("ast_hip::style_loss")
def _(x, y, weight, want_grad):
    b, c = x.shape[:2]
    if want_grad:
        return x.new_empty(()), x.new_empty((b, c, c)), x.new_empty((b * c,)), x.new_empty((b * c,))
    return x.new_empty(()), x.new_empty((0,)), x.new_empty((0,)), x.new_empty((0,))


def _style_setup(ctx, inputs, output):
    x, y, weight, want_grad = inputs
    if not want_grad:
        raise NotImplementedError("ast_hip::style_loss under autograd needs want_grad=True")
    ctx.save_for_backward(x, output[1], output[2], output[3])


def _style_backward(ctx, g, *_):
    x, dg, ra, rb = ctx.saved_tensors
    b, c, h, w = x.shape
    dx = torch.empty_like(x)
    check(lib().ast_gram_backward_f32(ptr(x), ptr(dg), ptr(dx), ptr(ra), ptr(rb), b, c, h * w, 1.0 / (c * h * w),
                                      ptr(g.contiguous()), 0, stream_ptr(x.device)), "gram_backward")
    return dx, None, None, None


register_autograd("ast_hip::style_loss", _style_backward, setup_context=_style_setup)


@custom_op("ast_hip::content_style_loss", mutates_args=())
def content_style_loss(x: Tensor, yc: Tensor, ys: Tensor, wc: float, ws: float,
                       want_grad: bool) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """(wc * content_mvn_loss(x, yc), ws * compute_style_loss(x, ys)) of ONE feature map x (the
    trainers apply both to every loss tap, train.py:217-245): the backward writes dx once -- the
    Gram-backward GEMM, then the content gradient added in place (the same fp32 sum autograd's add
    of the two gradients made, one read-modify-write of dx fewer). Extra outputs: the backward's
    state (pstats, dG, row_a, row_b; empty unless want_grad)."""
    n, c = x.shape[:2]
    acc_c, acc_s = _acc(x), _acc(x)
    pstats = torch.empty((n * c, 6), device=x.device) if want_grad else None
    Fn.mvn_huber(x, yc, wc, acc_c, pstats)
    dg, ra, rb = Fn._style_terms(x, ys, ws, acc_s, want_grad=want_grad)
    e = lambda t: t if t is not None else _empty(x)  # noqa: E731
    return acc_c[0], acc_s[0], e(pstats), e(dg), e(ra), e(rb)


@register_fake("ast_hip::content_style_loss")
def _(x, yc, ys, wc, ws, want_grad):
    b, c = x.shape[:2]
    if want_grad:
        return (x.new_empty(()), x.new_empty(()), x.new_empty((b * c, 6)), x.new_empty((b, c, c)),
                x.new_empty((b * c,)), x.new_empty((b * c,)))
    return (x.new_empty(()), x.new_empty(()), x.new_empty((0,)), x.new_empty((0,)), x.new_empty((0,)),
            x.new_empty((0,)))


def _cs_setup(ctx, inputs, output):
    x, yc, ys, wc, ws, want_grad = inputs
    if not want_grad:
        raise NotImplementedError("ast_hip::content_style_loss under autograd needs want_grad=True")
    ctx.save_for_backward(x, yc, output[2], output[3], output[4], output[5])
    ctx.wc = wc


def _cs_backward(ctx, gc, gs, *_):
    x, yc, pstats, dg, ra, rb = ctx.saved_tensors
    b, c, h, w = x.shape
    st = stream_ptr(x.device)
    dx = torch.empty_like(x)
    first = True
    if gs is not None:
        check(lib().ast_gram_backward_f32(ptr(x), ptr(dg), ptr(dx), ptr(ra), ptr(rb), b, c, h * w, 1.0 / (c * h * w),
                                          ptr(gs.contiguous()), 0, st), "gram_backward")
        first = False
    if gc is not None:
        check(lib().ast_mvn_huber_backward_f32(ptr(x), ptr(yc), ptr(pstats), b * c, h * w, ctx.wc,
                                               ptr(gc.contiguous()), ptr(dx), 0 if first else 1, st),
              "mvn_huber_backward")
        first = False
    if first:
        dx.zero_()
    return dx, None, None, None, None, None


register_autograd("ast_hip::content_style_loss", _cs_backward, setup_context=_cs_setup)


@custom_op("ast_hip::huber_loss", mutates_args=())
def huber_loss(x: Tensor, y: Tensor) -> Tensor:
    acc = _acc(x)
    check(lib().ast_huber_f32(ptr(x), ptr(y), x.numel(), 1.0, None, ptr(acc), None, 0, stream_ptr(x.device)), "huber")
    return acc[0]


@register_fake("ast_hip::huber_loss")
def _(x, y):
    return x.new_empty(())


def _huber_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[0], inputs[1])


def _huber_backward(ctx, g):
    x, y = ctx.saved_tensors
    g = g.contiguous()
    dx = dy = None
    if ctx.needs_input_grad[0]:
        dx = torch.empty_like(x)
        check(lib().ast_huber_f32(ptr(x), ptr(y), x.numel(), 1.0, ptr(g), None, ptr(dx), 0, stream_ptr(x.device)),
              "huber")
    if ctx.needs_input_grad[1]:
        dy = torch.empty_like(y)
        check(lib().ast_huber_f32(ptr(y), ptr(x), y.numel(), 1.0, ptr(g), None, ptr(dy), 0, stream_ptr(y.device)),
              "huber")
    return dx, dy


register_autograd("ast_hip::huber_loss", _huber_backward, setup_context=_huber_setup)


@custom_op("ast_hip::tv_loss", mutates_args=())
def tv_loss(img: Tensor) -> Tensor:
    n, c, h, w = img.shape
    acc = _acc(img)
    check(lib().ast_tv_loss_f32(ptr(img), n * c, h, w, 1.0, None, ptr(acc), None, 0, stream_ptr(img.device)),
          "tv_loss")
    return acc[0]


@register_fake("ast_hip::tv_loss")
def _(img):
    return img.new_empty(())


def _tv_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[0])


def _tv_backward(ctx, g):
    (img,) = ctx.saved_tensors
    n, c, h, w = img.shape
    dx = torch.empty_like(img)
    check(lib().ast_tv_loss_f32(ptr(img), n * c, h, w, 1.0, ptr(g.contiguous()), None, ptr(dx), 0,
                                stream_ptr(img.device)), "tv_loss")
    return dx


register_autograd("ast_hip::tv_loss", _tv_backward, setup_context=_tv_setup)


@custom_op("ast_hip::hist_loss", mutates_args=())
def hist_loss(x: Tensor, y: Tensor, weight: float) -> Tuple[Tensor, Tensor, Tensor]:
    """weight * compute_hist_loss(x, y); extra outputs: the two soft histograms."""
    hx, hy = Fn.soft_histogram(x), Fn.soft_histogram(y)
    acc = _acc(x)
    check(lib().ast_emd_loss_f32(ptr(hx), ptr(hy), x.shape[0], float(weight), None, ptr(acc), None,
                                 stream_ptr(x.device)), "emd_loss")
    return acc[0], hx, hy


@register_fake("ast_hip::hist_loss")
def _(x, y, weight):
    return x.new_empty(()), x.new_empty((x.shape[0], Fn.HIST_BINS)), x.new_empty((y.shape[0], Fn.HIST_BINS))


def _hist_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[0], output[1], output[2])
    ctx.weight = float(inputs[2])


def _hist_backward(ctx, g, *_):
    x, hx, hy = ctx.saved_tensors
    b = x.shape[0]
    ghist = torch.empty_like(hx)
    check(lib().ast_emd_loss_f32(ptr(hx), ptr(hy), b, ctx.weight, ptr(g.contiguous()), None, ptr(ghist),
                                 stream_ptr(x.device)), "emd_loss")
    dx = torch.empty_like(x)
    check(lib().ast_soft_hist_backward_f32(ptr(x), b, x.numel() // b, 1.0 / (x.shape[1] * x.shape[2]), ptr(ghist),
                                           ptr(dx), 0, stream_ptr(x.device)), "soft_hist_backward")
    return dx, None, None


register_autograd("ast_hip::hist_loss", _hist_backward, setup_context=_hist_setup)


@custom_op("ast_hip::range_loss", mutates_args=())
def range_loss(x: Tensor, weight: float) -> Tensor:
    acc = _acc(x)
    check(lib().ast_range_loss_f32(ptr(x), x.numel(), float(weight), None, ptr(acc), None, 0, stream_ptr(x.device)),
          "range_loss")
    return acc[0]


@register_fake("ast_hip::range_loss")
def _(x, weight):
    return x.new_empty(())


def _range_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[0])
    ctx.weight = float(inputs[1])


def _range_backward(ctx, g):
    (x,) = ctx.saved_tensors
    dx = torch.empty_like(x)
    check(lib().ast_range_loss_f32(ptr(x), x.numel(), ctx.weight, ptr(g.contiguous()), None, ptr(dx), 0,
                                   stream_ptr(x.device)), "range_loss")
    return dx, None


register_autograd("ast_hip::range_loss", _range_backward, setup_context=_range_setup)


@custom_op("ast_hip::sqdiff_mean", mutates_args=())
def sqdiff_mean(x: Tensor, y: Tensor, weight: float) -> Tensor:
    acc = _acc(x)
    check(lib().ast_sqdiff_mean_f32(ptr(x), ptr(y), x.numel(), float(weight), None, ptr(acc), None, 0,
                                    stream_ptr(x.device)), "sqdiff")
    return acc[0]


@register_fake("ast_hip::sqdiff_mean")
def _(x, y, weight):
    return x.new_empty(())


def _sqdiff_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[0], inputs[1])
    ctx.weight = float(inputs[2])


def _sqdiff_backward(ctx, g):
    x, y = ctx.saved_tensors
    dx = torch.empty_like(x)
    check(lib().ast_sqdiff_mean_f32(ptr(x), ptr(y), x.numel(), ctx.weight, ptr(g.contiguous()), None, ptr(dx), 0,
                                    stream_ptr(x.device)), "sqdiff")
    return dx, None, None


register_autograd("ast_hip::sqdiff_mean", _sqdiff_backward, setup_context=_sqdiff_setup)


# ------------------------------------------------------------------------------------------------
# MobileNet-variant inference ops (eval-mode BatchNorm folded into the weights)
# ------------------------------------------------------------------------------------------------

_DT = {torch.float32: 0, torch.bfloat16: 1}


@custom_op("ast_hip::mb_expand_dw", mutates_args=())
def mb_expand_dw(x: Tensor, x2: Optional[Tensor], w1p: Optional[Tensor], b1: Optional[Tensor], wdw: Tensor,
                 bdw: Tensor, hid: int, cin_pad: int, k: int, stride: int, up: int) -> Tuple[Tensor, Tensor]:
    """expand 1x1 (+ folded BN, Hardswish) -> depthwise kxk (reflect, + folded BN, Hardswish):
    the depthwise output D [n, hid, ho, wo] and the SE pool sums [n, hid]."""
    from .mobilenetv2 import _expand_dw
    n, c1, h, w = x.shape
    cin = c1 + (x2.shape[1] if x2 is not None else 0)
    p = (k - 1) // 2
    ho, wo = (h * up + 2 * p - k) // stride + 1, (w * up + 2 * p - k) // stride + 1
    d = torch.empty((n, hid, ho, wo), device=x.device, dtype=x.dtype)
    pool = torch.empty((n, hid), device=x.device, dtype=torch.float32)
    check(_expand_dw(x.dtype, x, x2, c1, n, cin, h, w, up, w1p, b1, hid, cin_pad, wdw, bdw, k, stride, d, pool, ho, wo,
                     stream_ptr(x.device)), "mb_expand_dw")
    return d, pool


@register_fake("ast_hip::mb_expand_dw")
def _(x, x2, w1p, b1, wdw, bdw, hid, cin_pad, k, stride, up):
    n, _, h, w = x.shape
    p = (k - 1) // 2
    ho, wo = (h * up + 2 * p - k) // stride + 1, (w * up + 2 * p - k) // stride + 1
    return x.new_empty((n, hid, ho, wo)), x.new_empty((n, hid), dtype=torch.float32)


@custom_op("ast_hip::mb_se_fold", mutates_args=())
def mb_se_fold(pool: Tensor, hw: int, fc1w: Tensor, fc1b: Tensor, fc2w: Tensor, fc2b: Tensor, w2: Tensor,
               cout_pad: int, hid_pad: int, bf16: bool) -> Tensor:
    """SELayer's MLP on the pooled means, its Hardtanh(0, 1) gate folded into the pw-linear weights:
    [n, cout_pad, hid_pad] (zero padded) in the activations' dtype."""
    n, hid = pool.shape
    cout = w2.shape[0]
    dt = torch.bfloat16 if bf16 else torch.float32
    wg = torch.empty((n, cout_pad, hid_pad), device=pool.device, dtype=dt)
    check(lib().ast_mb_se_fold(_DT[dt], ptr(pool), n, hid, hw, ptr(fc1w), ptr(fc1b), fc1w.shape[0], ptr(fc2w),
                               ptr(fc2b), ptr(w2), cout, cout_pad, hid_pad, ptr(wg), stream_ptr(pool.device)),
          "mb_se_fold")
    return wg


@register_fake("ast_hip::mb_se_fold")
def _(pool, hw, fc1w, fc1b, fc2w, fc2b, w2, cout_pad, hid_pad, bf16):
    return pool.new_empty((pool.shape[0], cout_pad, hid_pad), dtype=torch.bfloat16 if bf16 else torch.float32)


@custom_op("ast_hip::mb_pw", mutates_args=())
def mb_pw(d: Tensor, wg: Tensor, bias: Optional[Tensor], cout: int, res: Optional[Tensor], res_up: bool) -> Tensor:
    """pw-linear conv with the SE-gated weights (+ folded BN bias, + residual / upsampled residual)."""
    n, hid, h, w = d.shape
    cout_pad, hid_pad = wg.shape[1], wg.shape[2]
    out = torch.empty((n, cout, h, w), device=d.device, dtype=d.dtype)
    check(lib().ast_mb_pw(_DT[d.dtype], ptr(d), n, hid, hid_pad, h, w, ptr(wg), cout_pad * hid_pad, ptr(bias), cout,
                          cout_pad, ptr(res), 1 if res_up else 0, ptr(out), stream_ptr(d.device)), "mb_pw")
    return out


@register_fake("ast_hip::mb_pw")
def _(d, wg, bias, cout, res, res_up):
    return d.new_empty((d.shape[0], cout, d.shape[2], d.shape[3]))


@custom_op("ast_hip::mb_expand_gemm", mutates_args=())
def mb_expand_gemm(x: Tensor, x2: Optional[Tensor], w1p: Tensor, b1: Tensor, hid: int, cin_pad: int) -> Tensor:
    """The expand half of a wide DepthWiseConv (ada_out, 256 -> 768) as a GEMM + Hardswish."""
    n, c1, h, w = x.shape
    cin = c1 + (x2.shape[1] if x2 is not None else 0)
    out = torch.empty((n, hid, h, w), device=x.device, dtype=x.dtype)
    check(lib().ast_mb_expand_gemm(_DT[x.dtype], ptr(x), ptr(x2), c1, n, cin, h, w, ptr(w1p), ptr(b1), hid, cin_pad,
                                   ptr(out), stream_ptr(x.device)), "mb_expand_gemm")
    return out


@register_fake("ast_hip::mb_expand_gemm")
def _(x, x2, w1p, b1, hid, cin_pad):
    return x.new_empty((x.shape[0], hid, x.shape[2], x.shape[3]))


@custom_op("ast_hip::mb_conv3x3_dense", mutates_args=())
def mb_conv3x3_dense(x: Tensor, wt: Tensor, bias: Optional[Tensor], act: int, out_bf16: bool) -> Tensor:
    """Dense 3x3 reflect-pad conv of the variant (block 0 + Hardswish; the decoder image conv)."""
    n, cin, h, w = x.shape
    cout = wt.shape[0]
    dt = torch.bfloat16 if out_bf16 else torch.float32
    y = torch.empty((n, cout, h, w), device=x.device, dtype=dt)
    check(lib().ast_mb_conv3x3_dense(_DT[x.dtype], _DT[dt], ptr(x), ptr(wt), ptr(bias), ptr(y), n, cin, cout, h, w,
                                     act, stream_ptr(x.device)), "mb_conv3x3_dense")
    return y


@register_fake("ast_hip::mb_conv3x3_dense")
def _(x, wt, bias, act, out_bf16):
    return x.new_empty((x.shape[0], wt.shape[0], x.shape[2], x.shape[3]),
                       dtype=torch.bfloat16 if out_bf16 else torch.float32)


OPS: List[str] = ["conv3x3", "adain_map", "content_mvn_loss", "style_loss", "huber_loss", "tv_loss", "hist_loss",
                  "range_loss", "sqdiff_mean", "mb_expand_dw", "mb_se_fold", "mb_pw", "mb_expand_gemm",
                  "mb_conv3x3_dense"]
