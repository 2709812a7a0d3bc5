"""Training path of the MobileNet-variant modules (SURVEY.md §8f "next" #4: AutoEncoder training,
train_autoencoder.py:88-148) on the HIP kernels of csrc/mbtrain.hip.

The inference path (mobilenetv2.DepthWiseConv.run) folds eval-mode BatchNorm into the weights and
fuses whole blocks; training needs batch statistics and every intermediate, so here each layer of
a block's `_layers` (mobilenetv2.py:95-165, same order) is an autograd Function whose forward and
backward are HIP launches: 1x1 convs as MFMA GEMMs, depthwise convs, BatchNorm2d (training mode,
running statistics updated as torch does), Hardswish, SELayer, the residual add and the decoder's
nearest upsample. fp32 only (the reference trains in fp32).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from . import dp, ops
from ._lib import HipOpError, accumulator_pool, check, lib, ptr, stream_ptr, workspace
from .functional import _grad_buffer   # weight gradients straight into the DP / graph arena slice


def _s(t):
    return stream_ptr(t.device)


def _f32(t, name):
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise HipOpError(f"{name} must be a tensor on a HIP device")
    if t.dtype != torch.float32:
        raise HipOpError(f"{name}: the training path runs in float32, got {t.dtype}")
    return t.contiguous()


_AUTOSPLIT = os.environ.get("AST_MBGEMM_AUTOSPLIT", "1") != "0"


def gemm(A, B, C, M, N, K, batch, sA, sB, sC, ksplit=1, accumulate=False, fold_k=0, fold_n=0, role=""):
    """C[b][m][n] (+)= sum_k A[b][m][k] B[b][k][n]; sA/sB/sC = (batch, row, col) element strides.
    fold_n / fold_k = P: the image index is folded into N / K (batch 1; see ast_hip.h). K-split or
    batch-shared C tiles meet in a workspace and are summed in a fixed order (deterministic).
    A product with fewer than 256 64x64 tiles (the AST bottleneck's 1x1 convs at 20x20: 26-100
    workgroups on 256 CUs) and K >= 128 is split along K to ~512 workgroups, chunks >= 64 deep
    (AST_MBGEMM_AUTOSPLIT=0: off, for A/B runs)."""
    if _AUTOSPLIT and ksplit == 1 and not fold_k:
        tiles = -(-M // 64) * -(-N // 64) * batch
        if tiles < 256 and K >= 128:
            ksplit = max(1, min(-(-512 // tiles), K // 64))
            # the C side rounds the chunk up to a multiple of 32 (GK): recount the splits so none is empty
            kchunk = -(-(-(-K // ksplit)) // 32) * 32
            ksplit = -(-K // kchunk)
    nws = int(lib().ast_mbt_gemm_workspace_floats(M, N, batch, ksplit, sC[0]))
    ws = workspace(nws, C.device) if nws > 0 else None
    check(ops._timed(f"mbgemm {role} {M}x{N}x{K}", 2 * M * N * K * batch, C.device, lambda: lib().ast_mbt_gemm_f32(
        ptr(A), ptr(B), ptr(C), M, N, K, batch, *sA, *sB, *sC, ksplit, int(accumulate), fold_k, fold_n, ptr(ws),
        nws, _s(C))), "gemm")


def _ksplit(m, n, k):
    """Split the weight gradient's long reduction so ~1024 workgroups run (4 per CU), chunks >= 256
    deep; the partial tiles meet in the workspace and are summed in split order."""
    tiles = -(-m // 64) * -(-n // 64)
    return max(1, min(-(-1024 // tiles), k // 256, 65535))


# ------------------------------------------------------------------------------------------------
# 1x1 conv (no bias), optionally over a channel-split input (the un-materialised torch.cat)
# ------------------------------------------------------------------------------------------------
class PwConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, x2, weight):
        x = _f32(x, "x")
        n, c1, h, w = x.shape
        P = h * w
        cout, cin = weight.shape[0], weight.shape[1]
        wt = weight.detach().reshape(cout, cin).contiguous()
        y = torch.empty((n, cout, h, w), device=x.device, dtype=torch.float32)
        gemm(wt, x, y, cout, n * P, c1, 1, (0, cin, 1), (c1 * P, P, 1), (cout * P, P, 1), fold_n=P, role="fwd")
        if x2 is not None:
            x2 = _f32(x2, "x2")
            c2 = x2.shape[1]
            gemm(wt[:, c1:], x2, y, cout, n * P, c2, 1, (0, cin, 1), (c2 * P, P, 1), (cout * P, P, 1), accumulate=True,
                 fold_n=P, role="fwd")
        ctx.save_for_backward(x, x2 if x2 is not None else x, wt)
        ctx.has_x2 = x2 is not None
        ctx.wshape = weight.shape
        ctx.param = weight
        return y

    @staticmethod
    def backward(ctx, g):
        x, x2, wt = ctx.saved_tensors
        g = _f32(g, "grad")
        n, cout, h, w = g.shape
        P = h * w
        cin = wt.shape[1]
        c1 = x.shape[1]
        dx = dx2 = dw = None
        parts = [(x, 0)] + ([(x2, c1)] if ctx.has_x2 else [])
        grads = []
        for xi, off in parts:
            ci = xi.shape[1]
            d = None
            if ctx.needs_input_grad[0 if off == 0 else 1]:
                d = torch.empty_like(xi)
                gemm(wt[:, off:], g, d, ci, n * P, cout, 1, (0, 1, cin), (cout * P, P, 1), (ci * P, P, 1),
                     fold_n=P, role="dgrad")
            grads.append(d)
        dx = grads[0]
        if ctx.has_x2:
            dx2 = grads[1]
        if ctx.needs_input_grad[2]:
            dw = _grad_buffer(ctx.param, ctx.wshape, g).view(cout, cin)
            for xi, off in parts:
                ci = xi.shape[1]
                gemm(g, xi, dw[:, off:], cout, ci, n * P, 1, (cout * P, P, 1), (ci * P, 1, P), (0, cin, 1),
                     ksplit=_ksplit(cout, ci, n * P), fold_k=P, role="wgrad")
            dw = dw.reshape(ctx.wshape)
        return dx, dx2, dw


class DwConvFn(torch.autograd.Function):
    """Depthwise k x k conv, stride s, reflect padding (k-1)/2. act = 1: the conv's input is
    hardswish(x), x the pre-activation (the block's Hardswish fused into the staging; the backward
    returns the gradient w.r.t. x)."""

    @staticmethod
    def forward(ctx, x, weight, k, s, act=0):
        x = _f32(x, "x")
        n, c, h, w = x.shape
        p = (k - 1) // 2
        ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
        wt = weight.detach().reshape(c, k * k).contiguous()
        y = torch.empty((n, c, ho, wo), device=x.device, dtype=torch.float32)
        check(lib().ast_mbt_dw_act_f32(0, ptr(x), ptr(wt), None, ptr(y), n, c, h, w, k, s, int(act), None, 0, _s(x)),
              "dw conv")
        ctx.save_for_backward(x, wt)
        ctx.k, ctx.s, ctx.act, ctx.wshape = k, s, int(act), weight.shape
        ctx.param = weight
        return y

    @staticmethod
    def backward(ctx, g):
        x, wt = ctx.saved_tensors
        g = _f32(g, "grad")
        n, c, h, w = x.shape
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            check(lib().ast_mbt_dw_act_f32(1, ptr(x) if ctx.act else None, ptr(wt), ptr(g), ptr(dx), n, c, h, w, ctx.k,
                                           ctx.s, ctx.act, None, 0, _s(g)), "dw dgrad")
        if ctx.needs_input_grad[1]:
            dw = _grad_buffer(ctx.param, ctx.wshape, g).view(c, ctx.k * ctx.k)
            ws = workspace(lib().ast_mbt_dw_workspace_floats(n, c, h, w, ctx.k), x.device)
            check(lib().ast_mbt_dw_act_f32(2, ptr(x), ptr(wt), ptr(g), ptr(dw), n, c, h, w, ctx.k, ctx.s, ctx.act,
                                           ptr(ws), ws.numel(), _s(g)), "dw wgrad")
            dw = dw.reshape(ctx.wshape)
        return dx, dw, None, None, None


# BatchNorm's num_batches_tracked bookkeeping (torch increments it on every train-mode forward): a
# trainer step defers the increments and applies them as one multi-tensor add at its end (one launch
# instead of one per BatchNorm call: 84 per ASTTrainer step); outside a step each call adds at once.
_BN_PENDING = None


def _bump_batches_tracked(bn):
    if _BN_PENDING is None:
        bn.num_batches_tracked.add_(1)
    else:
        t = bn.num_batches_tracked
        _BN_PENDING[id(t)] = (t, _BN_PENDING.get(id(t), (t, 0))[1] + 1)


class deferred_bn_counters:
    """Context of one training step: the num_batches_tracked increments of every train-mode
    BatchNorm call inside it become one torch._foreach_add_ on exit (a BatchNorm run twice in the
    step -- the AST encoder over the content and over the stylised image -- counts twice)."""

    def __enter__(self):
        global _BN_PENDING
        self.prev, _BN_PENDING = _BN_PENDING, {}
        self.pool = accumulator_pool().__enter__()   # and the step's loss accumulators, pooled
        return self

    def __exit__(self, *exc):
        global _BN_PENDING
        try:
            self.pool.__exit__(*exc)
        finally:
            pend, _BN_PENDING = _BN_PENDING, self.prev
        if pend and exc[0] is None:   # a step that raised did not complete its forward: no count
            ts = [t for t, _ in pend.values()]
            torch._foreach_add_(ts, [k for _, k in pend.values()])


def _bn_workspace(x, n, c, hw):
    return torch.empty((max(1, lib().ast_mbt_bn_workspace_floats(n, c, hw)),), device=x.device, dtype=torch.float32)


class BatchNormTrainFn(torch.autograd.Function):
    """BatchNorm2d.forward in training mode (batch statistics; running stats updated in place),
    with `act` = 1 the following Hardswish fused in (DepthWiseConv's BN -> Hardswish pairs,
    mobilenetv2.py:122-126, :150-153): one apply pass writes hardswish(BN(x)), and the backward
    takes the Hardswish derivative at the recomputed BN output inside its two passes (the BN output
    is never stored). A BatchNorm marked by dp.convert_sync_batchnorm takes its statistics over
    every rank's images (all-gather of per-rank (count, mean, M2), all-reduce of the backward sums)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, bn, act=0):
        x = _f32(x, "x")
        n, c, h, w = x.shape
        mean = torch.empty((c,), device=x.device, dtype=torch.float32)
        invstd = torch.empty_like(mean)
        y = torch.empty_like(x)
        ws = _bn_workspace(x, n, c, h * w)
        track = bn.track_running_stats and bn.running_mean is not None
        momentum = bn.momentum if bn.momentum is not None else 0.1
        rm = ptr(bn.running_mean) if track else None
        rv = ptr(bn.running_var) if track else None
        group = dp.sync_group(bn)
        ctx.group, ctx.act = group, int(act)
        inv_count = None
        if group is None:
            check(lib().ast_mbt_bn_act_fwd_f32(ptr(x), n, c, h * w, ptr(gamma), ptr(beta), float(bn.eps),
                                               float(momentum), ptr(mean), ptr(invstd), rm, rv, ctx.act, ptr(y),
                                               ptr(ws), ws.numel(), _s(x)), "batch norm")
        else:
            L = lib()
            stats = torch.empty((c, 3), device=x.device, dtype=torch.float64)
            check(L.ast_mbt_bn_stats_f32(ptr(x), n, c, h * w, ptr(ws), ws.numel(), ptr(stats), _s(x)), "bn stats")
            allst = dp.all_gather_bn_stats(stats, group)
            inv_count = torch.empty((1,), device=x.device, dtype=torch.float32)
            check(L.ast_mbt_bn_merge_f32(ptr(allst), allst.shape[0], c, float(bn.eps), float(momentum), ptr(mean),
                                         ptr(invstd), rm, rv, ptr(inv_count), _s(x)), "bn merge")
            check(L.ast_mbt_bn_act_apply_f32(ptr(x), n, c, h * w, ptr(mean), ptr(invstd), ptr(gamma), ptr(beta),
                                             ctx.act, ptr(y), _s(x)), "bn apply")
        if track:
            _bump_batches_tracked(bn)   # bookkeeping counter (torch does the same increment)
        ctx.save_for_backward(x, gamma, beta, mean, invstd, inv_count if inv_count is not None else mean)
        ctx.params = (gamma, beta)
        return y

    @staticmethod
    def backward(ctx, g):
        x, gamma, beta, mean, invstd, inv_count = ctx.saved_tensors
        g = _f32(g, "grad")
        n, c, h, w = x.shape
        dx = torch.empty_like(x)
        ws = _bn_workspace(x, n, c, h * w)
        if ctx.group is None:
            dgamma = _grad_buffer(ctx.params[0], (c,), mean)
            dbeta = _grad_buffer(ctx.params[1], (c,), mean)
            check(lib().ast_mbt_bn_act_bwd_f32(ptr(x), ptr(g), n, c, h * w, ptr(mean), ptr(invstd), ptr(gamma),
                                               ptr(beta), ctx.act, ptr(dgamma), ptr(dbeta), ptr(dx), ptr(ws),
                                               ws.numel(), _s(g)), "batch norm backward")
            return dx, dgamma, dbeta, None, None
        L = lib()
        sums = torch.empty((2, c), device=x.device, dtype=torch.float32)
        check(L.ast_mbt_bn_act_bwd_sums_f32(ptr(x), ptr(g), n, c, h * w, ptr(mean), ptr(invstd), ptr(gamma),
                                            ptr(beta), ctx.act, ptr(ws), ws.numel(), ptr(sums), _s(g)),
              "bn backward sums")
        dgamma = _grad_buffer(ctx.params[0], (c,), mean)
        dbeta = _grad_buffer(ctx.params[1], (c,), mean)
        dbeta.copy_(sums[0])      # local: the gradient all-reduce averages them
        dgamma.copy_(sums[1])
        dp.all_reduce_sum(sums, ctx.group)
        check(L.ast_mbt_bn_act_bwd_apply_f32(ptr(x), ptr(g), n, c, h * w, ptr(mean), ptr(invstd), ptr(gamma),
                                             ptr(beta), ctx.act, ptr(sums), ptr(inv_count), ptr(dx), _s(g)),
              "bn backward apply")
        return dx, dgamma, dbeta, None, None


class HardswishFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = _f32(x, "x")
        y = torch.empty_like(x)
        check(lib().ast_mbt_eltwise_f32(0, ptr(x), None, ptr(y), x.numel(), 0, 0, _s(x)), "hardswish")
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        dx = torch.empty_like(x)
        check(lib().ast_mbt_eltwise_f32(1, ptr(x), ptr(_f32(g, "grad")), ptr(dx), x.numel(), 0, 0, _s(x)),
              "hardswish backward")
        return dx


class AddFn(torch.autograd.Function):
    """The residual `x + org_x` (mobilenetv2.py:162-163)."""

    @staticmethod
    def forward(ctx, a, b):
        a, b = _f32(a, "a"), _f32(b, "b")
        y = torch.empty_like(a)
        check(lib().ast_mbt_eltwise_f32(2, ptr(a), ptr(b), ptr(y), a.numel(), 0, 0, _s(a)), "add")
        return y

    @staticmethod
    def backward(ctx, g):
        return g, g


class Upsample2Fn(torch.autograd.Function):
    """nn.Upsample(scale_factor=2, mode="nearest") (models.py:266)."""

    @staticmethod
    def forward(ctx, x):
        x = _f32(x, "x")
        n, c, h, w = x.shape
        y = torch.empty((n, c, 2 * h, 2 * w), device=x.device, dtype=torch.float32)
        check(lib().ast_mbt_eltwise_f32(3, ptr(x), None, ptr(y), n * c, h, w, _s(x)), "upsample")
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, g):
        n, c, h, w = ctx.shape
        dx = torch.empty(ctx.shape, device=g.device, dtype=torch.float32)
        check(lib().ast_mbt_eltwise_f32(4, ptr(_f32(g, "grad")), None, ptr(dx), n * c, h, w, _s(g)), "upsample bwd")
        return dx


class SEFn(torch.autograd.Function):
    """SELayer.forward (mobilenetv2.py:72-81): x * Hardtanh(0,1)(fc2(relu(fc1(avgpool(x))))).
    act = 1: the SE input is hardswish(x), x the pre-activation (the block's Hardswish fused into
    the pool and scale passes; the backward returns the gradient w.r.t. x)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, act=0):
        x = _f32(x, "x")
        n, c, h, w = x.shape
        red = w1.shape[0]
        act = int(act)
        pool = torch.empty((n, c), device=x.device, dtype=torch.float32)
        L = lib()
        check(L.ast_mbt_plane_act_f32(3 if act else 0, ptr(x), None, None, None, None, ptr(pool), n * c, h * w, _s(x)),
              "se pool")
        hid = torch.empty((n, red), device=x.device, dtype=torch.float32)
        z = torch.empty((n, c), device=x.device, dtype=torch.float32)
        gate = torch.empty_like(z)
        w1c, w2c = w1.detach().contiguous(), w2.detach().contiguous()
        check(L.ast_mbt_se_fc_fwd_f32(ptr(pool), ptr(w1c), ptr(b1), ptr(w2c), ptr(b2), n, c, red, ptr(hid), ptr(z),
                                      ptr(gate), _s(x)), "se fc")
        y = torch.empty_like(x)
        check(L.ast_mbt_plane_act_f32(5 if act else 2, ptr(x), None, ptr(gate), None, None, ptr(y), n * c, h * w,
                                      _s(x)), "se scale")
        ctx.save_for_backward(x, w1c, w2c, pool, hid, z, gate)
        ctx.act = act
        ctx.params = (w1, b1, w2, b2)
        return y

    @staticmethod
    def backward(ctx, g):
        x, w1, w2, pool, hid, z, gate = ctx.saved_tensors
        g = _f32(g, "grad")
        n, c, h, w = x.shape
        red = w1.shape[0]
        L = lib()
        dgate = torch.empty((n, c), device=x.device, dtype=torch.float32)
        check(L.ast_mbt_plane_act_f32(4 if ctx.act else 1, ptr(g), ptr(x), None, None, None, ptr(dgate), n * c, h * w,
                                      _s(g)), "se dgate")
        pw1, pb1, pw2, pb2 = ctx.params
        dw1, db1 = _grad_buffer(pw1, tuple(w1.shape), x), _grad_buffer(pb1, (red,), x)
        dw2, db2 = _grad_buffer(pw2, tuple(w2.shape), x), _grad_buffer(pb2, (c,), x)
        dpool = torch.empty((n, c), device=x.device, dtype=torch.float32)
        ws = workspace(n * (c + red), x.device)
        check(L.ast_mbt_se_fc_bwd_f32(ptr(dgate), ptr(z), ptr(hid), ptr(pool), ptr(w1), ptr(w2), n, c, red, h * w,
                                      ptr(dw1), ptr(db1), ptr(dw2), ptr(db2), ptr(dpool), ptr(ws), ws.numel(), _s(g)),
              "se fc bwd")
        dx = torch.empty_like(x)
        check(L.ast_mbt_plane_act_f32(6 if ctx.act else 2, ptr(g), None, ptr(gate), ptr(dpool),
                                      ptr(x) if ctx.act else None, ptr(dx), n * c, h * w, _s(g)), "se dx")
        return dx, dw1, db1, dw2, db2, None


# BatchNorm -> Hardswish, Hardswish -> depthwise conv and Hardswish -> SELayer run fused (no
# materialised activation); AST_MBT_FUSE=0: the unfused layer chain (A/B runs, bit-identical)
_FUSE_BN_ACT = os.environ.get("AST_MBT_FUSE", "1") != "0"


def block_forward(block, x, x2=None, up: int = 1):
    """DepthWiseConv.forward (mobilenetv2.py:153-165) layer by layer, BatchNorm in the module's
    mode (training: batch statistics). `up` applies DecoderBlock's nearest upsample first."""
    if x.dtype != torch.float32:
        raise HipOpError("the MobileNet training path runs in float32")
    if up == 2:
        x = Upsample2Fn.apply(x)
    org_x = x
    h = x
    first_conv = True
    layers = list(block._layers)
    skip = False
    pending_act = 0   # a Hardswish carried into the next depthwise conv / SELayer (not materialised)
    for i, layer in enumerate(layers):
        if skip:   # the Hardswish fused into the BatchNorm before it
            skip = False
            continue
        if isinstance(layer, nn.ReflectionPad2d):
            continue  # the ratio-1 block's pad: the depthwise kernel pads reflect by (k-1)/2 = 1
        if isinstance(layer, nn.Conv2d):
            if layer.groups > 1:
                k = layer.kernel_size[0]
                h = DwConvFn.apply(h, layer.weight, k, layer.stride[0], pending_act)
                pending_act = 0
            else:
                h = PwConvFn.apply(h, x2 if first_conv else None, layer.weight)
            first_conv = False
        elif isinstance(layer, nn.BatchNorm2d):
            if layer.training:
                act = int(i + 1 < len(layers) and isinstance(layers[i + 1], nn.Hardswish) and _FUSE_BN_ACT)
                h = BatchNormTrainFn.apply(h, layer.weight, layer.bias, layer, act)
                skip = bool(act)
            else:
                raise NotImplementedError("eval-mode BatchNorm under autograd: use the inference path "
                                          "(torch.no_grad()) or train mode")
        elif isinstance(layer, nn.Hardswish):
            nxt = layers[i + 1] if i + 1 < len(layers) else None
            if _FUSE_BN_ACT and (nxt.__class__.__name__ == "SELayer" or
                                 (isinstance(nxt, nn.Conv2d) and nxt.groups > 1)):
                pending_act = 1
            else:
                h = HardswishFn.apply(h)
        elif layer.__class__.__name__ == "SELayer":
            fc1, fc2 = layer.fc[0], layer.fc[2]
            h = SEFn.apply(h, fc1.weight, fc1.bias, fc2.weight, fc2.bias, pending_act)
            pending_act = 0
        else:
            raise NotImplementedError(f"layer {layer.__class__.__name__} in the training path")
    if block.identity:
        h = AddFn.apply(h, org_x)
    return h


def wants_training_path(module, *xs) -> bool:
    """True when a forward must record autograd through the HIP training kernels."""
    if not torch.is_grad_enabled():
        return False
    return any(p.requires_grad for p in module.parameters()) or any(
        x is not None and x.requires_grad for x in xs)
