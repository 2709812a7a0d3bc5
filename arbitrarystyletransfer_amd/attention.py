"""AdaAttN (models.py:70-115) with a HIP backward, for training the reference's own AST model
(train.py:146-300 trains `self.ast.parameters()`, which include ada_att_1 / ada_att_2).

Forward: ops.adaattn (one fused flash-style launch; the Nq x Nk attention matrix never leaves
registers). Backward: the attention is recomputed per image with the batched MFMA GEMMs of
csrc/mbtrain.hip (`ast_mbt_gemm_f32`, strided operands, fp32 as the reference trains) and the
elementwise / row-reduction stages of csrc/adaattn_bwd.hip; the derivation is in that file's head.
Two forms of the attention part of the backward:
  * materialised (small maps): P and dS as [n][Nq][Nk] fp32 through the batched GEMMs -- 5 MB at the
    reference's 160^2 training images (20^2 maps, B=8), where full-width GEMM tiles win;
  * flash (csrc/adaattn_flash.hip; round 4), once P would reach FLASH_MIN_BYTES (64 MiB: 64^2 maps
    at one image): the scores are recomputed per 16 x 16 block in registers by three passes (row
    statistics; dK and d[V; V^2] per key; dQ per query) and neither P nor dS is ever stored -- they
    grow as (H W)^2, 1 GB per image at 128^2 maps. AST_ADAATTN_FLASH=1|0 forces one form.
"""
from __future__ import annotations

import os

import torch

from . import ops
from ._lib import HipOpError, check, lib, ptr, stream_ptr
from .functional import _grad_buffer
from .mbtrain import gemm


def _s(t):
    return stream_ptr(t.device)


def _in_stats(x):
    """InstanceNorm2d (models.py:77-79: affine=False, eps 1e-5, biased variance): mean, std, x_hat."""
    m, s = ops.channel_stats(x, unbiased=False, eps=1e-5)
    return m, s, ops.plane_normalize(x, m, s)


FLASH_MIN_BYTES = 64 << 20


def use_flash(n, C, N, M) -> bool:
    """Whether AdaAttNFn.backward takes the flash form (see the module docstring)."""
    env = os.environ.get("AST_ADAATTN_FLASH")
    if env == "0" or not lib().ast_adaattn_flash_supported(int(C)):
        return False
    return env == "1" or 4 * n * N * M >= FLASH_MIN_BYTES


def _wsplit(n, k):
    """K split of the weight-gradient GEMMs (reduction over images x pixels) for ~1024 workgroups."""
    return max(1, min(1024 // max(1, n * 4), k // 256, 65535))


class AdaAttNFn(torch.autograd.Function):
    """out = AdaAttN(c, s; W_q, W_k, W_v); gradients for all five (fp32)."""

    @staticmethod
    def forward(ctx, c, s, wq, wk, wv):
        out = ops.adaattn(c, s, wq, wk, wv)
        ctx.save_for_backward(c, s, wq, wk, wv)
        ctx.params = (wq, wk, wv)
        return out

    @staticmethod
    def backward(ctx, g):
        c, s, wq, wk, wv = ctx.saved_tensors
        if c.dtype != torch.float32:
            raise HipOpError("AdaAttN backward runs in float32 (the reference trains in fp32)")
        g = ops._dev(g, "grad")
        n, C, hc, wc = (int(v) for v in c.shape)
        hs, ws_ = int(s.shape[2]), int(s.shape[3])
        N, M = hc * wc, hs * ws_
        dev = c.device
        f = lambda *shape: torch.empty(shape, device=dev, dtype=torch.float32)  # noqa: E731
        L = lib()
        st = _s(c)
        Wq, Wk, Wv = (w.detach().float().reshape(C, C).contiguous() for w in (wq, wk, wv))
        mc, sc, chat = _in_stats(c)
        ms, ss, shat = _in_stats(s)
        Q, K, VV = f(n, C, N), f(n, C, M), f(n, 2 * C, M)
        gemm(Wq, chat, Q, C, N, C, n, (0, C, 1), (C * N, N, 1), (C * N, N, 1), role="attn q")
        gemm(Wk, shat, K, C, M, C, n, (0, C, 1), (C * M, M, 1), (C * M, M, 1), role="attn k")
        gemm(Wv, s, VV, C, M, C, n, (0, C, 1), (C * M, M, 1), (2 * C * M, M, 1), role="attn v")
        check(L.ast_adaattn_square_f32(ptr(VV), n, C * M, st), "adaattn_square")
        flash = use_flash(n, C, N, M)
        O2 = f(n, N, 2 * C)
        if flash:
            lse2 = f(n, N)
            check(L.ast_adaattn_flash_stats_f32(ptr(Q), ptr(K), ptr(VV), ptr(O2), ptr(lse2), n, C, N, M, st),
                  "adaattn_flash_stats")
        else:
            P = f(n, N, M)
            gemm(Q, K, P, N, M, C, n, (C * N, 1, N), (C * M, M, 1), (N * M, M, 1), role="attn s")
            check(L.ast_softmax_rows_f32(ptr(P), n * N, M, st), "softmax_rows")
            gemm(P, VV, O2, N, 2 * C, M, n, (N * M, M, 1), (2 * C * M, 1, M), (N * 2 * C, 2 * C, 1), role="attn o")
        dO2, D = f(n, N, 2 * C), f(n * N)
        need_dc = ctx.needs_input_grad[0]
        std = f(n, C, N) if need_dc else None
        check(L.ast_adaattn_dstats_f32(ptr(O2), ptr(g), ptr(chat), ptr(dO2), ptr(D), ptr(std), n, C, N, st),
              "adaattn_dstats")
        dVV = f(n, 2 * C, M)
        dQ, dK = f(n, C, N), f(n, C, M)
        if flash:
            check(L.ast_adaattn_flash_bwd_kv_f32(ptr(Q), ptr(K), ptr(VV), ptr(dO2), ptr(lse2), ptr(D), ptr(dK),
                                                 ptr(dVV), n, C, N, M, st), "adaattn_flash_bwd_kv")
            check(L.ast_adaattn_flash_bwd_q_f32(ptr(Q), ptr(K), ptr(VV), ptr(dO2), ptr(lse2), ptr(D), ptr(dQ),
                                                n, C, N, M, st), "adaattn_flash_bwd_q")
        else:
            dS = f(n, N, M)
            gemm(dO2, VV, dS, N, M, 2 * C, n, (N * 2 * C, 2 * C, 1), (2 * C * M, M, 1), (N * M, M, 1), role="attn dp")
            check(L.ast_softmax_backward_f32(ptr(P), ptr(dS), ptr(D), n * N, M, st), "softmax_backward")
            gemm(dO2, P, dVV, 2 * C, M, N, n, (N * 2 * C, 1, 2 * C), (N * M, M, 1), (2 * C * M, M, 1), role="attn dvv")
            gemm(K, dS, dQ, C, N, M, n, (C * M, M, 1), (N * M, 1, M), (C * N, N, 1), role="attn dq")
            gemm(Q, dS, dK, C, M, N, n, (C * N, N, 1), (N * M, M, 1), (C * M, M, 1), role="attn dk")
            del P, dS
        dV = f(n, C, M)
        check(L.ast_adaattn_dv_f32(ptr(dVV), ptr(VV), ptr(dV), n, C * M, st), "adaattn_dv")
        grads = [None] * 5
        for i, (dX, Xh, P_) in ((2, (dQ, chat, N)), (3, (dK, shat, M)), (4, (dV, s, M))):
            if ctx.needs_input_grad[i]:
                wp = ctx.params[i - 2]
                dW = _grad_buffer(wp, tuple(wp.shape), dX) if wp.dtype == torch.float32 else f(C, C)
                gemm(dX, Xh, dW.view(C, C), C, C, P_, n, (C * P_, P_, 1), (C * P_, 1, P_), (0, C, 1),
                     ksplit=_wsplit(n, P_), role="attn dw")
                grads[i] = dW.view_as(wp).to(wp.dtype)
        if need_dc:
            dchat = f(n, C, N)
            gemm(Wq, dQ, dchat, C, N, C, n, (0, 1, C), (C * N, N, 1), (C * N, N, 1), role="attn dchat")
            check(L.ast_fma_inplace_f32(ptr(dchat), ptr(g), ptr(std), n * C * N, st), "fma")
            dc = torch.empty_like(c)
            check(L.ast_instance_norm_backward_f32(ptr(c), ptr(mc), ptr(sc), ptr(dchat), ptr(dc), n * C, N, 0, st),
                  "instance_norm_backward")
            grads[0] = dc
        if ctx.needs_input_grad[1]:
            ds = f(n, C, M)
            gemm(Wv, dV, ds, C, M, C, n, (0, 1, C), (C * M, M, 1), (C * M, M, 1), role="attn ds")
            dshat = f(n, C, M)
            gemm(Wk, dK, dshat, C, M, C, n, (0, 1, C), (C * M, M, 1), (C * M, M, 1), role="attn dshat")
            check(L.ast_instance_norm_backward_f32(ptr(s), ptr(ms), ptr(ss), ptr(dshat), ptr(ds), n * C, M, 1, st),
                  "instance_norm_backward")
            grads[1] = ds.view_as(s)
        return tuple(grads)


def adaattn(module, content_map, style_map):
    """AdaAttN forward with autograd (the training path of models.AdaAttN)."""
    for name, t in (("content_map", content_map), ("style_map", style_map)):
        if t.dtype != torch.float32:
            raise HipOpError(f"AdaAttN training runs in float32; {name} is {t.dtype}")
    return AdaAttNFn.apply(content_map.contiguous(), style_map.contiguous(), module.W_q.weight, module.W_k.weight,
                           module.W_v.weight)
