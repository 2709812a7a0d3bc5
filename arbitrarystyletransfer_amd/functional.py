"""Autograd for the HIP ops: torch.autograd.Function wrappers whose forward and backward are
both HIP kernels of libast_hip.so, so `loss.backward()` in a train.py-style loop runs the
backward on the GPU through the same C ABI (no PyTorch compute on the path).
"""
from __future__ import annotations

import os

import torch

from . import ops
from ._lib import HipOpError, check, lib, loss_accumulator, ptr, stream_ptr, workspace

_dev = ops._dev


def _s(t):
    return stream_ptr(t.device)


def _empty(shape, like):
    return torch.empty(shape, device=like.device, dtype=torch.float32)


# ------------------------------------------------------------------------------------------------
# weight packs for the backward (cached per parameter version)
# ------------------------------------------------------------------------------------------------

class TFPackCache:
    """Transposed+flipped weight packs (input-gradient filters), refreshed on parameter change.

    The pack is stored on the parameter itself (`_ast_tf_pack`), so its lifetime follows the
    tensor: a freed model's packs go with it, and a new parameter that reuses a dead one's
    address can never hit a stale entry."""

    def get(self, weight: torch.Tensor, in_scale=None) -> torch.Tensor:
        w = _dev(weight.detach(), "weight")
        key = (weight.data_ptr(), weight._version, ops.weight_epoch(weight),
               None if in_scale is None else (in_scale.data_ptr(), in_scale._version))
        hit = getattr(weight, "_ast_tf_pack", None)
        if hit is not None and hit[0] == key:
            return hit[1]
        cout, cin = int(w.shape[0]), int(w.shape[1])
        out = torch.empty(int(lib().ast_conv3x3_packed_numel(cin, cout)), device=w.device, dtype=torch.float32)
        check(lib().ast_conv3x3_pack_weights_ex_f32(ptr(w), ptr(out), cout, cin, 1, ptr(in_scale), _s(w)),
              "pack_weights_ex")
        weight._ast_tf_pack = (key, out)
        return out


_TF = TFPackCache()


def conv_input_grad_same(dy, weight, in_scale=None):
    """Gradient of conv3x3(x, zero pad) wrt x, given dL/dy (same-size transposed conv)."""
    cout, cin = int(weight.shape[0]), int(weight.shape[1])
    pre, _, _ = ops.conv3x3(dy, _TF.get(weight, in_scale), None, cin, pad_mode="zeros",
                            want_pre=True, want_act=False)
    return pre


_E_UNSUPPORTED = -3  # AST_E_UNSUPPORTED (include/ast_hip.h)


def dgrad_kind(up):
    """conv_tuning.json key suffix of an ast_conv3x3_dgrad_f32 launch (scripts/tune_conv.py TUNE_DGRAD)."""
    return " dgrad sum2" if up == 2 else " dgrad"


def conv_input_grad(dy, weight, upsample=1, pad_mode="zeros", in_scale=None, mask=None, add_pre=None,
                    add_post=None):
    """dL/dx of y = conv3x3(pad(upsample(x))) given dL/dy, with the fused input-gradient epilogue of
    ast_conv3x3_dgrad_f32: dx = mask > 0 ? add_post + (g + add_pre) : add_post (mask = the ReLU
    output feeding this conv: the ReLU backward of the layer below; add_pre / add_post = gradient
    taps of that layer's ReLU output / pre-ReLU output; each optional). Reflect padding: the
    border fold (ast_dgrad_reflect_border_f32) after the interior. Configurations without the
    fused epilogue (small packed planes, cin < 16 after the swap) run the plain input-gradient conv
    and the same epilogue as one elementwise pass (identical arithmetic per element)."""
    dy = _dev(dy, "dy")
    cout, cin = int(weight.shape[0]), int(weight.shape[1])
    n, _, H, W = (int(v) for v in dy.shape)
    up = int(upsample)
    h, w = H // up, W // up
    ext = []
    for t, name in ((mask, "mask"), (add_pre, "add_pre"), (add_post, "add_post")):
        if t is not None:
            t = _dev(t, name)
            if tuple(t.shape) != (n, cin, h, w):
                raise HipOpError(f"{name} {tuple(t.shape)} must be the input's shape {(n, cin, h, w)}")
        ext.append(t)
    mask, add_pre, add_post = ext
    if pad_mode == "reflect" and in_scale is not None:
        raise HipOpError("in_scale (the conv_1 normalisation) comes with zero padding only")
    if up == 1 and mask is None and add_pre is None and add_post is None:
        dx = conv_input_grad_same(dy, weight, in_scale)
    else:
        dx = _empty((n, cin, h, w), dy)
        code = _E_UNSUPPORTED
        if ops.pack_plan(n, W, False) == (1, 0):
            packed = _TF.get(weight, in_scale)
            cfg = ops.tuned_config(n, cout, H, W, cin, 1, "zeros", False, dgrad_kind(up))
            code = ops._timed(f"conv3x3 dgrad {cout}->{cin} {H}x{W} up{up}", 2 * n * H * W * cout * cin * 9, dy.device,
                              lambda: lib().ast_conv3x3_dgrad_f32(cfg, ptr(dy), ptr(packed), ptr(dx), ptr(mask),
                                                                  ptr(add_pre), ptr(add_post), n, cout, H, W, cin,
                                                                  up, _s(dy)))
        if code == _E_UNSUPPORTED:
            raw = conv_input_grad_same(dy, weight, in_scale)
            check(lib().ast_dgrad_finish_f32(ptr(raw), ptr(dx), ptr(mask), ptr(add_pre), ptr(add_post), n * cin, h, w,
                                             up, _s(dy)), "dgrad_finish")
        else:
            check(code, "conv3x3_dgrad")
    if pad_mode == "reflect":
        wt = _dev(weight.detach(), "weight")
        ws = workspace(lib().ast_dgrad_reflect_border_workspace_floats(n, cout, cin, h, w, up), dy.device)
        check(lib().ast_dgrad_reflect_border_f32(ptr(dy), ptr(wt), ptr(dx), ptr(mask), ptr(ws), ws.numel(), n, cout,
                                                 cin, h, w, up, _s(dy)), "dgrad_reflect_border")
    return dx


# id(parameter) -> dp.FlatGradArena: weight gradients are written straight into the arena slice
# (a view, which autograd adopts as .grad without copying).
GRAD_ARENA = {}


def _grad_buffer(param, shape, like):
    """Output buffer of a weight-gradient kernel (which overwrites it). The arena slice is handed
    out at most once per backward (dp.FlatGradArena.take): a parameter used twice in the graph
    (the decoder under full_losses runs on t and on f_c) gets a fresh buffer for its second
    contribution, which autograd then sums with the first, instead of both contributions being
    written into -- and wiping -- the same storage."""
    arena = GRAD_ARENA.get(id(param)) if param is not None else None
    if arena is not None:
        view = arena.take(param)
        if view is not None:
            return view
    return _empty(shape, like)


def conv_weight_grad(x, dy, cout, upsample=1, pad_mode="zeros", with_bias=True, weight=None, bias=None,
                     dy_layout=(0, 0, 0)):
    """dW, db of conv3x3(pad(upsample(x))); dy dense [n, cout, H, W] or, with dy_layout =
    (pitch, plane, offset), the padded gradient buffer of the decoder dgrad."""
    x = _dev(x, "x")
    dy = _dev(dy, "dy")
    n, cin, h, w = (int(s) for s in x.shape)
    dw = _grad_buffer(weight, (cout, cin, 3, 3), x)
    db = _grad_buffer(bias, (cout,), x) if with_bias else None
    flops = 2 * n * h * upsample * w * upsample * cout * cin * 9
    pitch, plane, off = dy_layout
    ws = workspace(lib().ast_conv3x3_wgrad_workspace_floats(n, cin, h, w, cout, upsample), x.device)
    check(ops._timed(f"wgrad {cin}->{cout} {h * upsample}x{w * upsample}", flops, x.device,
                     lambda: lib().ast_conv3x3_wgrad_ex_f32(ptr(x), ptr(dy), ptr(dw), ptr(db), n, cin, h, w, cout,
                                                            upsample, ops.PAD_MODES[pad_mode], pitch, plane, off,
                                                            ptr(ws), ws.numel(), _s(x))),
          "conv3x3_wgrad")
    return dw, db


# ------------------------------------------------------------------------------------------------
# VGG encoder block: conv3x3 (zero pad) -> {pre, ReLU, ReLU+MaxPool} (PretrainedEncoder)
# ------------------------------------------------------------------------------------------------

class EncoderConvFn(torch.autograd.Function):
    """Outputs (pre, act, pool) — the conv_i / relu_i / pool_i taps; unrequested ones are empty
    tensors. `norm` = (mean, std) for conv_1 (Normalization fused into the gather)."""

    @staticmethod
    def forward(ctx, x, weight, bias, packed, want_act, want_pool, mean, std):
        ctx.set_materialize_grads(False)
        pre, act, pool = ops.conv3x3(x, packed, bias, weight.shape[0], pad_mode="zeros", in_mean=mean,
                                     in_std=std, want_pre=True, want_act=want_act, want_pool=want_pool)
        ctx.save_for_backward(x, weight, pre, mean, std)
        ctx.has_bias = bias is not None
        ctx.param_ids = (weight, bias)
        e = x.new_empty(0)
        return pre, (act if act is not None else e), (pool if pool is not None else e)

    @staticmethod
    def backward(ctx, g_pre, g_act, g_pool):
        x, weight, pre, mean, std = ctx.saved_tensors
        n, cout, h, w = pre.shape
        gp = g_pre if (g_pre is not None and g_pre.numel()) else None
        ga = g_act if (g_act is not None and g_act.numel()) else None
        gq = g_pool if (g_pool is not None and g_pool.numel()) else None
        dy = torch.empty_like(pre)
        check(lib().ast_conv_act_backward_f32(ptr(pre), ptr(_dev(gp, "g") if gp is not None else None),
                                              ptr(_dev(ga, "g") if ga is not None else None),
                                              ptr(_dev(gq, "g") if gq is not None else None), ptr(dy),
                                              n * cout, h, w, _s(pre)), "conv_act_backward")
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = conv_input_grad_same(dy, weight, std.view(-1) if std is not None else None)
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            xin = x
            if mean is not None:  # conv_1 sees the normalised image
                xin = normalize_image(x, mean, std)
            dw, db = conv_weight_grad(xin, dy, cout, with_bias=ctx.has_bias, weight=ctx.param_ids[0],
                                      bias=ctx.param_ids[1])
        return dx, dw, db, None, None, None, None, None


class LossNetFn(torch.autograd.Function):
    """The whole frozen VGG walk of PretrainedEncoder (models.py:226-240) as one autograd node, so
    its backward sees every tap gradient at once and can fuse across layers: the ReLU backward of a
    layer not followed by a max-pool runs in the next layer's input-gradient epilogue (mask = that
    conv's input, the ReLU output; the layer's relu_i / conv_i tap gradients as add_pre / add_post,
    conv_input_grad), instead of a separate ast_conv_act_backward_f32 pass per layer. Layers under a
    max-pool and the top layer keep that pass (it routes the pooled gradient). Same arithmetic per
    element as the per-layer EncoderConvFn chain. Used when no conv parameter needs a gradient
    (the loss network of every trainer); forward outputs: the requested taps in network order."""

    @staticmethod
    def forward(ctx, net, x):
        ctx.set_materialize_grads(False)
        norm = net._vgg_layers[0]
        plan = net._plan()
        outs, pres, ins = [], [], []
        cur = x
        for k, (idx, conv, want_pre, want_act, want_pool, collect) in enumerate(plan):
            first = idx == 1
            # the pre-ReLU map is kept only where the backward reads it: under a max-pool (argmax
            # routing) and at the top layer; elsewhere the next conv's input (the ReLU output) is the
            # mask, so a layer without a conv_i tap stores its ReLU output alone
            keep_pre = want_pre or want_pool or k == len(plan) - 1
            pre, act, pool = ops.conv3x3(cur, net._packed.get(conv), conv.bias, conv.out_channels, pad_mode="zeros",
                                         in_mean=norm.mean.view(-1) if first else None,
                                         in_std=norm.std.view(-1) if first else None,
                                         want_pre=keep_pre, want_act=want_act, want_pool=want_pool)
            by_name = {conv.name: pre, f"relu_{idx}": act, f"pool_{idx}": pool}
            outs.extend(by_name[nm] for nm in collect)
            pres.append(pre)
            ins.append(cur)
            cur = pool if want_pool else act
        ctx.plan = [(idx, conv, want_pool, collect) for idx, conv, _, _, want_pool, collect in plan]
        ctx.std = norm.std.view(-1)
        ctx.save_for_backward(*pres, *ins[1:])
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        saved = ctx.saved_tensors
        L = len(ctx.plan)
        pres, ins = saved[:L], (None,) + tuple(saved[L:])
        taps, k = [], 0
        for idx, conv, want_pool, collect in ctx.plan:
            t = {}
            for nm in collect:
                t[nm.split("_")[0]] = grads[k]
                k += 1
            taps.append((t.get("conv"), t.get("relu"), t.get("pool")))

        def act_backward(j, g_pool):
            gp, ga, gq = taps[j]
            if g_pool is not None:
                gq = g_pool if gq is None else gq + g_pool
            if gp is None and ga is None and gq is None:
                return None
            # act > 0 exactly where pre > 0: a layer without a stored pre-ReLU map (no pool below it)
            # masks by its ReLU output, the next conv's input
            pre = pres[j] if pres[j] is not None else ins[j + 1]
            n, c, h, w = pre.shape
            dy = torch.empty_like(pre)
            check(lib().ast_conv_act_backward_f32(ptr(pre), ptr(_dev(gp, "g") if gp is not None else None),
                                                  ptr(_dev(ga, "g") if ga is not None else None),
                                                  ptr(_dev(gq, "g") if gq is not None else None), ptr(dy),
                                                  n * c, h, w, _s(pre)), "conv_act_backward")
            return dy

        dy = act_backward(L - 1, None)
        for j in range(L - 1, 0, -1):
            conv = ctx.plan[j][1]
            pooled = ctx.plan[j - 1][2]
            if dy is None:
                dy = act_backward(j - 1, None)
            elif pooled:
                dy = act_backward(j - 1, conv_input_grad(dy, conv.weight))
            else:
                gp, ga, _ = taps[j - 1]
                dy = conv_input_grad(dy, conv.weight, mask=ins[j], add_pre=ga, add_post=gp)
        dx = None
        if dy is not None and ctx.needs_input_grad[1]:
            dx = conv_input_grad(dy, ctx.plan[0][1].weight, in_scale=ctx.std)
        return None, dx


def normalize_image(x, mean, std):
    x = _dev(x, "x")
    n, c = x.shape[:2]
    out = torch.empty_like(x)
    m = mean.reshape(-1).repeat(n).contiguous()
    s = std.reshape(-1).repeat(n).contiguous()
    check(lib().ast_plane_normalize_f32(ptr(x), ptr(m), ptr(s), ptr(out), n * c, x[0, 0].numel(), _s(x)),
          "normalize")
    return out


# ------------------------------------------------------------------------------------------------
# Decoder block: [Upsample x2] -> ReflectionPad(1) -> conv3x3 -> [ReLU]
# ------------------------------------------------------------------------------------------------

class DecoderConvFn(torch.autograd.Function):
    """[Upsample x2] -> ReflectionPad(1) -> conv3x3 -> [ReLU] (models.py:598-628).

    Backward: dy = the output gradient (ReLU-masked here unless `out_premasked`), then the input
    gradient with the reflect border fold (conv_input_grad) and the weight gradient on dense dy.
    `mask_input`: the input is the ReLU output of the previous decoder layer and feeds only this
    layer, so that layer's ReLU backward (input > 0) runs in this layer's input-gradient epilogue;
    the previous layer is then built with `out_premasked` and passes its gradient through."""

    @staticmethod
    def forward(ctx, x, weight, bias, packed, upsample, relu, mask_input=False, out_premasked=False):
        pre, act, _ = ops.conv3x3(x, packed, bias, weight.shape[0], upsample=upsample, pad_mode="reflect",
                                  want_pre=not relu, want_act=relu)
        out = act if relu else pre
        ctx.save_for_backward(x, weight, out)
        ctx.upsample, ctx.relu, ctx.has_bias = upsample, relu, bias is not None
        ctx.mask_input, ctx.out_premasked = bool(mask_input), bool(out_premasked)
        ctx.param_ids = (weight, bias)  # for the DP gradient arena lookup (not saved tensors)
        return out

    @staticmethod
    def backward(ctx, g):
        x, weight, out = ctx.saved_tensors
        g = _dev(g, "grad")
        n, cout, H, W = out.shape
        if ctx.relu and not ctx.out_premasked:
            dy = torch.empty_like(g)
            check(lib().ast_relu_mask_f32(ptr(g), ptr(out), ptr(dy), g.numel(), _s(g)), "relu_mask")
        else:
            dy = g
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = conv_input_grad(dy, weight, ctx.upsample, "reflect", mask=x if ctx.mask_input else None)
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            dw, db = conv_weight_grad(x, dy, cout, ctx.upsample, "reflect", ctx.has_bias, *ctx.param_ids)
        return (dx, dw, db) + (None,) * (len(ctx.needs_input_grad) - 3)  # 6 or 8 inputs


# ------------------------------------------------------------------------------------------------
# Statistics / AdaIN
# ------------------------------------------------------------------------------------------------

class ChannelStatsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, unbiased, eps):
        mean, std = ops.channel_stats(x, unbiased, eps)
        ctx.save_for_backward(x, mean, std)
        ctx.unbiased = unbiased
        return mean, std

    @staticmethod
    def backward(ctx, dmean, dstd):
        x, mean, std = ctx.saved_tensors
        x = _dev(x, "x")
        n, c = x.shape[:2]
        dx = torch.empty_like(x)
        dm = _dev(dmean, "dmean") if dmean is not None else None
        ds = _dev(dstd, "dstd") if dstd is not None else None
        check(lib().ast_channel_stats_backward_f32(ptr(x), ptr(mean), ptr(std), ptr(dm), ptr(ds), ptr(dx), n * c,
                                                   x[0, 0].numel(), 1 if ctx.unbiased else 0, 0, _s(x)),
              "channel_stats_backward")
        return dx, None, None


class MeanVarianceNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return ops.mean_variance_norm(x)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        x = _dev(x, "x")
        g = _dev(g, "grad")
        n, c = x.shape[:2]
        dx = torch.empty_like(x)
        check(lib().ast_mvn_backward_f32(ptr(x), ptr(g), ptr(dx), n * c, x[0, 0].numel(), 1e-5, _s(x)),
              "mvn_backward")
        return dx


class AdaINFn(torch.autograd.Function):
    """AdaIN (models.py:43-51) + alpha blend (models.py:471), HIP forward and backward."""

    @staticmethod
    def forward(ctx, content, style, alpha, swap):
        ctx.save_for_backward(content, style)
        ctx.alpha, ctx.swap = alpha, swap
        return ops.adain(content, style, alpha=alpha, swap_style_stats=swap)

    @staticmethod
    def backward(ctx, g):
        content, style = ctx.saved_tensors
        content, style = _dev(content, "content"), _dev(style, "style")
        g = _dev(g, "grad")
        n, c, hc, wc = content.shape
        hs, ws = style.shape[2:]
        dc = torch.empty_like(content) if ctx.needs_input_grad[0] else None
        ds = torch.empty_like(style) if ctx.needs_input_grad[1] else None
        if dc is None and ds is None:
            return None, None, None, None
        check(lib().ast_adain_backward_f32(ptr(content), ptr(style), ptr(g), ptr(dc), ptr(ds), n, c, hc, wc, hs, ws,
                                           float(ctx.alpha), 1 if ctx.swap else 0, _s(g)), "adain_backward")
        return dc, ds, None, None


def channel_stats(x, unbiased=True, eps=0.0):
    if torch.is_grad_enabled() and x.requires_grad:
        return ChannelStatsFn.apply(x, unbiased, eps)
    return ops.channel_stats(x, unbiased, eps)


def mean_variance_norm(x):
    if torch.is_grad_enabled() and x.requires_grad:
        return MeanVarianceNormFn.apply(x)
    return ops.mean_variance_norm(x)


# ------------------------------------------------------------------------------------------------
# Losses (scalar outputs; the backward kernels take grad_output as a device scalar)
# ------------------------------------------------------------------------------------------------

def _acc(like):
    """A loss accumulator (ast_hip.h: value at [0], then the per-workgroup partials that the
    kernels sum in a fixed order)."""
    return loss_accumulator(like.device)


def _value(acc):
    """The 0-d loss value of an accumulator (a view of element 0)."""
    return acc[0]


def gram(f, g, scale):
    """g[b] = scale * f[b] f[b]^T for f [b, c, hw] (the deterministic split-K launch)."""
    b, c = int(f.shape[0]), int(f.shape[1])
    hw = f.numel() // (b * c)
    ws = workspace(lib().ast_gram_workspace_floats(b, c, hw), f.device)
    check(ops._timed(f"gram {c}x{hw}", 2 * b * c * c * hw, f.device,
                     lambda: lib().ast_gram_f32(ptr(f), ptr(g), b, c, hw, scale, ptr(ws), ws.numel(), _s(f))), "gram")


class GramFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f):
        f = _dev(f, "tensor")
        b, c, h, w = f.shape
        g = _empty((b, c, c), f)
        gram(f, g, 1.0 / (c * h * w))
        ctx.save_for_backward(f)
        return g

    @staticmethod
    def backward(ctx, dg):
        (f,) = ctx.saved_tensors
        b, c, h, w = f.shape
        dg = _dev(dg, "grad")
        df = torch.empty_like(f)
        check(lib().ast_gram_backward_f32(ptr(f), ptr(dg), ptr(df), None, None, b, c, h * w, 1.0 / (c * h * w),
                                          None, 0, _s(f)), "gram_backward")
        return df


class HuberFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y):
        x, y = _dev(x, "input"), _dev(y, "target")
        if x.shape != y.shape:
            raise HipOpError(f"huber: shape mismatch {tuple(x.shape)} vs {tuple(y.shape)}")
        loss = _acc(x)
        check(lib().ast_huber_f32(ptr(x), ptr(y), x.numel(), 1.0, None, ptr(loss), None, 0, _s(x)), "huber")
        ctx.save_for_backward(x, y)
        return _value(loss)

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        g = _dev(g, "grad")
        dx = dy = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            check(lib().ast_huber_f32(ptr(x), ptr(y), x.numel(), 1.0, ptr(g), None, ptr(dx), 0, _s(x)), "huber")
        if ctx.needs_input_grad[1]:
            dy = torch.empty_like(y)
            check(lib().ast_huber_f32(ptr(y), ptr(x), y.numel(), 1.0, ptr(g), None, ptr(dy), 0, _s(y)), "huber")
        return dx, dy


# the content / style-moment losses' split-plane launches (AST_PLANE_SPLIT=0: one workgroup per
# plane, the round-2 kernels; kept for A/B measurement)
PLANE_SPLIT = os.environ.get("AST_PLANE_SPLIT", "1") == "1"


def mvn_huber(x, y, weight, loss, pstats):
    """loss += weight * compute_content_loss(mvn(x), mvn(y)); pstats (or None) for the backward.
    The split-plane launch (chunk partials merged in order through a workspace)."""
    n, c = int(x.shape[0]), int(x.shape[1])
    hw = x[0, 0].numel()
    if not PLANE_SPLIT:
        check(lib().ast_mvn_huber_f32(ptr(x), ptr(y), n * c, hw, weight, ptr(loss), ptr(pstats), _s(x)), "mvn_huber")
        return
    ws = workspace(lib().ast_plane_stats_workspace_floats(n * c, hw), x.device)
    check(lib().ast_mvn_huber_ws_f32(ptr(x), ptr(y), n * c, hw, weight, ptr(loss), ptr(pstats), ptr(ws), ws.numel(),
                                     _s(x)), "mvn_huber")


class MVNHuberFn(torch.autograd.Function):
    """compute_content_loss(mean_variance_norm(x), mean_variance_norm(y)) with y detached (as
    every call site in train.py), one fused kernel for value and gradient."""

    @staticmethod
    def forward(ctx, x, y, weight):
        x, y = _dev(x, "x"), _dev(y, "y")
        if x.shape != y.shape:
            raise HipOpError(f"content loss: shape mismatch {tuple(x.shape)} vs {tuple(y.shape)}")
        n, c = x.shape[:2]
        loss = _acc(x)
        pstats = _empty((n * c, 6), x) if ctx.needs_input_grad[0] else None
        mvn_huber(x, y, weight, loss, pstats)
        ctx.save_for_backward(x, y, pstats)
        ctx.weight = weight
        return _value(loss)

    @staticmethod
    def backward(ctx, g):
        x, y, pstats = ctx.saved_tensors
        g = _dev(g, "grad")
        n, c = x.shape[:2]
        dx = torch.empty_like(x)
        check(lib().ast_mvn_huber_backward_f32(ptr(x), ptr(y), ptr(pstats), n * c, x[0, 0].numel(), ctx.weight,
                                               ptr(g), ptr(dx), 0, _s(x)), "mvn_huber_backward")
        return dx, None, None


class StyleLossFn(torch.autograd.Function):
    """compute_style_loss(x, y) (losses.py:128-139) with y detached: value in forward; the
    backward recomputes the statistics and Gram matrices and emits dx in two launches
    (moment terms fused into the Gram-backward GEMM epilogue)."""

    @staticmethod
    def forward(ctx, x, y, weight):
        x, y = _dev(x, "x"), _dev(y, "y")
        if x.shape[:2] != y.shape[:2]:
            raise HipOpError("style loss: (N, C) mismatch")
        loss = _acc(x)
        # with a gradient to come, the forward also keeps dG and the moment-term coefficients
        # (all linear in grad_output), so the backward is one GEMM with grad_output as a scale
        dg, ra, rb = _style_terms(x, y, weight, loss, want_grad=ctx.needs_input_grad[0])
        ctx.save_for_backward(x, dg, ra, rb)
        return _value(loss)

    @staticmethod
    def backward(ctx, g):
        x, dg, ra, rb = ctx.saved_tensors
        b, c, h, w = x.shape
        dx = torch.empty_like(x)
        gg = _dev(g, "grad")
        check(ops._timed(f"gram_bwd {c}x{h * w}", 2 * b * c * c * h * w, x.device,
                         lambda: lib().ast_gram_backward_f32(ptr(x), ptr(dg), ptr(dx), ptr(ra), ptr(rb), b, c, h * w,
                                                             1.0 / (c * h * w), ptr(gg), 0, _s(x))), "gram_backward")
        return dx, None, None


def _style_terms(x, y, weight, loss, want_grad):
    """Value of weight * compute_style_loss(x, y) added into `loss`; with want_grad also
    (dG, row_a, row_b) of its gradient for grad_output = 1."""
    b, c, h, w = x.shape
    hw = h * w
    planes = b * c
    stats = _empty((planes, 4), x)
    ra = _empty((planes,), x) if want_grad else None
    rb = _empty((planes,), x) if want_grad else None
    L = lib()
    s = _s(x)
    if y.shape[2:] != x.shape[2:]:
        raise HipOpError("style loss: feature maps must have the same spatial size")
    if not PLANE_SPLIT:
        check(L.ast_style_moments_f32(ptr(x), ptr(y), planes, hw, weight, None, ptr(stats), ptr(loss), ptr(ra),
                                      ptr(rb), s), "style_moments")
    else:
        ws = workspace(L.ast_plane_stats_workspace_floats(planes, hw), x.device)
        check(L.ast_style_moments_ws_f32(ptr(x), ptr(y), planes, hw, weight, None, ptr(stats), ptr(loss), ptr(ra),
                                         ptr(rb), ptr(ws), ws.numel(), s), "style_moments")
    gx = _empty((b, c, c), x)
    gy = _empty((b, c, c), x)
    scale = 1.0 / (c * hw)
    gram(x, gx, scale)
    gram(y, gy, scale)
    dg = _empty((b, c, c), x) if want_grad else None
    check(L.ast_gram_huber_f32(ptr(gx), ptr(gy), b * c * c, weight, None, ptr(loss), ptr(dg), s), "gram_huber")
    return dg, ra, rb


class TVLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img):
        img = _dev(img, "img")
        n, c, h, w = img.shape
        loss = _acc(img)
        check(lib().ast_tv_loss_f32(ptr(img), n * c, h, w, 1.0, None, ptr(loss), None, 0, _s(img)), "tv_loss")
        ctx.save_for_backward(img)
        return _value(loss)

    @staticmethod
    def backward(ctx, g):
        (img,) = ctx.saved_tensors
        n, c, h, w = img.shape
        dx = torch.empty_like(img)
        check(lib().ast_tv_loss_f32(ptr(img), n * c, h, w, 1.0, ptr(_dev(g, "grad")), None, ptr(dx), 0, _s(img)),
              "tv_loss")
        return dx


# ------------------------------------------------------------------------------------------------
# Histogram / range / pixel losses (train.py:255-269; SURVEY.md §8f "next" #2)
# ------------------------------------------------------------------------------------------------

HIST_BINS = 256   # HistLayerBase.K, losses.py:44


def soft_histogram(x):
    """SingleDimHistLayer.forward (losses.py:52-57) of x [B, C, H, W] (or [B, C, H]):
    [B, 256], normalised by C*H as the reference (x.size(1) * x.size(2))."""
    x = _dev(x, "x")
    b = x.shape[0]
    hist = _empty((b, HIST_BINS), x)
    ws = workspace(lib().ast_soft_hist_workspace_floats(b), x.device)
    check(lib().ast_soft_hist_f32(ptr(x), b, x.numel() // b, 1.0 / (x.shape[1] * x.shape[2]), ptr(hist), ptr(ws),
                                  ws.numel(), _s(x)), "soft_hist")
    return hist


class HistLossFn(torch.autograd.Function):
    """weight * compute_hist_loss(x, y) (losses.py:84-87): EMD between the soft histograms of x
    and y, mean over the batch; y is data (no gradient), as at train.py:261."""

    @staticmethod
    def forward(ctx, x, y, weight):
        x, y = _dev(x, "t_cs"), _dev(y, "style_map")
        if x.shape[0] != y.shape[0]:
            raise HipOpError(f"hist loss: batch mismatch {tuple(x.shape)} vs {tuple(y.shape)}")
        hx, hy = soft_histogram(x), soft_histogram(y)
        loss = _acc(x)
        check(lib().ast_emd_loss_f32(ptr(hx), ptr(hy), x.shape[0], float(weight), None, ptr(loss), None, _s(x)),
              "emd_loss")
        ctx.save_for_backward(x, hx, hy)
        ctx.weight = float(weight)
        return _value(loss)

    @staticmethod
    def backward(ctx, g):
        x, hx, hy = ctx.saved_tensors
        g = _dev(g, "grad")
        b = x.shape[0]
        ghist = torch.empty_like(hx)
        check(lib().ast_emd_loss_f32(ptr(hx), ptr(hy), b, ctx.weight, ptr(g), None, ptr(ghist), _s(x)), "emd_loss")
        dx = torch.empty_like(x)
        check(lib().ast_soft_hist_backward_f32(ptr(x), b, x.numel() // b, 1.0 / (x.shape[1] * x.shape[2]),
                                               ptr(ghist), ptr(dx), 0, _s(x)), "soft_hist_backward")
        return dx, None, None


class RangeLossFn(torch.autograd.Function):
    """weight * compute_content_loss(x, torch.clip(x.detach(), 0, 1)) (train.py:259)."""

    @staticmethod
    def forward(ctx, x, weight):
        x = _dev(x, "x")
        loss = _acc(x)
        check(lib().ast_range_loss_f32(ptr(x), x.numel(), float(weight), None, ptr(loss), None, 0, _s(x)),
              "range_loss")
        ctx.save_for_backward(x)
        ctx.weight = float(weight)
        return _value(loss)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        dx = torch.empty_like(x)
        check(lib().ast_range_loss_f32(ptr(x), x.numel(), ctx.weight, ptr(_dev(g, "grad")), None, ptr(dx), 0, _s(x)),
              "range_loss")
        return dx, None


class SqDiffMeanFn(torch.autograd.Function):
    """weight * ((y - x) ** 2).mean() with y constant (train.py:268: content_imgs.detach())."""

    @staticmethod
    def forward(ctx, x, y, weight):
        x, y = _dev(x, "x"), _dev(y, "y")
        if x.shape != y.shape:
            raise HipOpError(f"sqdiff: shape mismatch {tuple(x.shape)} vs {tuple(y.shape)}")
        loss = _acc(x)
        check(lib().ast_sqdiff_mean_f32(ptr(x), ptr(y), x.numel(), float(weight), None, ptr(loss), None, 0, _s(x)),
              "sqdiff")
        ctx.save_for_backward(x, y)
        ctx.weight = float(weight)
        return _value(loss)

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        dx = torch.empty_like(x)
        check(lib().ast_sqdiff_mean_f32(ptr(x), ptr(y), x.numel(), ctx.weight, ptr(_dev(g, "grad")), None, ptr(dx), 0,
                                        _s(x)), "sqdiff")
        return dx, None, None
