"""Drop-in for the reference losses.py: gram_matrix, compute_content_loss, compute_style_loss,
tv_loss and the soft-histogram / Earth-Mover loss compute_hist_loss
(losses.py:8-87; §8f "next" #2), with the SingleDimHistLayer / EarthMoversDistanceLoss modules
and the module-level `hist` / `earth_movers` instances. Every loss is a torch.ops.ast_hip custom op
(library.py) whose forward and backward are HIP kernels: one fused launch for the value, one for
the gradient."""
from __future__ import annotations

from . import functional as Fn
from . import library  # noqa: F401  (registers torch.ops.ast_hip.*)
from .ops import _dev

import torch
import torch.nn as nn

_ops = torch.ops.ast_hip


def _grad(x):
    return torch.is_grad_enabled() and x.requires_grad


class _SymmetricLoss(torch.autograd.Function):
    """A loss symmetric in its two arguments (L(x, y) = L(y, x): Huber of differences of the two
    sides' statistics, the EMD of their histograms) differentiated in BOTH, as the reference's own
    losses are (losses.py:84-87, 124-139 differentiate the target too). The value is fn(x, y); the
    backward recomputes fn(x, y) for x's gradient and fn(y, x) for y's, through the ops' own HIP
    backward kernels. Only a grad-requiring target takes this path; every reference caller detaches
    it (train.py:225-277), and those calls keep the one-sided fused op."""

    @staticmethod
    def forward(ctx, x, y, fn):
        ctx.fn = fn
        ctx.save_for_backward(x, y)
        return fn(x, y)

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        grads = [None, None]
        with torch.enable_grad():
            for i, (a, b) in enumerate(((x, y), (y, x))):
                if ctx.needs_input_grad[i]:
                    ar = a.detach().requires_grad_(True)
                    grads[i], = torch.autograd.grad(ctx.fn(ar, b.detach()), ar, g)
        return grads[0], grads[1], None


def _two_sided(fn, x, y):
    if torch.is_grad_enabled() and y.requires_grad:
        return _SymmetricLoss.apply(x, y, fn)
    return fn(x, y.detach())


def _pair(x, y, what):
    x, y = _dev(x, "input"), _dev(y, "target")
    if x.shape != y.shape:
        raise Fn.HipOpError(f"{what}: shape mismatch {tuple(x.shape)} vs {tuple(y.shape)}")
    return x, y

__all__ = ["gram_matrix", "compute_content_loss", "compute_style_loss", "tv_loss", "compute_hist_loss",
           "content_mvn_loss", "style_loss_weighted", "content_style_loss", "EarthMoversDistanceLoss",
           "HistLayerBase",
           "SingleDimHistLayer", "hist", "earth_movers", "out_of_range_loss", "pixel_mse_loss"]


def gram_matrix(tensor):
    """losses.py:105-109: bmm(F, F^T) / (C*H*W), F = tensor.view(B, C, H*W)."""
    return _ops.gram(_dev(tensor, "tensor"))


def compute_content_loss(inp, tgt):
    """losses.py:124-126: F.huber_loss(inp, tgt) (delta 1, mean)."""
    return _ops.huber_loss(*_pair(inp, tgt, "huber"))


def compute_style_loss(t_cs_map, style_map):
    """losses.py:128-139: 1.25*huber(mean) + 1.25*huber(std) + 10*huber(gram), differentiable in
    both arguments as the reference (train.py:233 passes style_map[i].detach(): then only t_cs_map)."""
    x, y = _dev(t_cs_map, "x"), _dev(style_map, "y")
    if x.shape[:2] != y.shape[:2] or x.shape[2:] != y.shape[2:]:
        raise Fn.HipOpError(f"style loss: shape mismatch {tuple(x.shape)} vs {tuple(y.shape)}")
    return _two_sided(lambda a, b: _ops.style_loss(a, b, 1.0, _grad(a))[0], x, y)


def tv_loss(img):
    """losses.py:90-103: sum of squared horizontal and vertical neighbour differences."""
    return _ops.tv_loss(_dev(img, "img"))


def content_mvn_loss(inp, tgt, weight: float = 1.0):
    """weight * compute_content_loss(mean_variance_norm(inp), mean_variance_norm(tgt.detach()))
    in one fused kernel (train.py:223-227, 258, 277)."""
    x, y = _pair(inp, tgt.detach(), "content loss")
    return _ops.content_mvn_loss(x, y, float(weight), _grad(x))[0]


def content_style_loss(inp, content_tgt, style_tgt, content_weight: float = 1.0, style_weight: float = 1.0):
    """(content_weight * content_mvn_loss(inp, content_tgt), style_weight * compute_style_loss(inp,
    style_tgt)) -- the pair the trainers take at every loss tap (train.py:217-245, 258, 271), with
    the input gradient formed in one buffer (library.content_style_loss)."""
    x = _dev(inp, "x")
    yc, ys = _dev(content_tgt.detach(), "content target"), _dev(style_tgt.detach(), "style target")
    if x.shape != yc.shape or x.shape != ys.shape:
        raise Fn.HipOpError(f"content/style loss: shape mismatch {tuple(x.shape)} vs {tuple(yc.shape)}, "
                            f"{tuple(ys.shape)}")
    out = _ops.content_style_loss(x, yc, ys, float(content_weight), float(style_weight), _grad(x))
    return out[0], out[1]


def style_loss_weighted(t_cs_map, style_map, weight: float = 1.0):
    """weight * compute_style_loss(t_cs_map, style_map.detach()) (train.py:230-245, 271)."""
    x, y = _dev(t_cs_map, "x"), _dev(style_map.detach(), "y")
    if x.shape[:2] != y.shape[:2] or x.shape[2:] != y.shape[2:]:
        raise Fn.HipOpError(f"style loss: shape mismatch {tuple(x.shape)} vs {tuple(y.shape)}")
    return _ops.style_loss(x, y, float(weight), _grad(x))[0]


class EarthMoversDistanceLoss(nn.Module):
    """losses.py:8-22: per-row sum of squared CDF differences of (Batch x Bins) inputs."""

    def forward(self, x, y):
        from .ops import emd_rows
        return emd_rows(x, y)


class HistLayerBase(nn.Module):
    """losses.py:40-48: K = 256 bins of width L = 1/K on [0, 1], sigmoid sharpness W = L/2.5."""

    def __init__(self):
        super().__init__()
        self.K = Fn.HIST_BINS
        self.L = 1 / self.K
        self.W = self.L / 2.5


class SingleDimHistLayer(HistLayerBase):
    """losses.py:51-57: one soft histogram over all values of each image, / (x.size(1)*x.size(2))."""

    def forward(self, x):
        return Fn.soft_histogram(x)


hist = SingleDimHistLayer()                # losses.py:79
earth_movers = EarthMoversDistanceLoss()   # losses.py:80


def compute_hist_loss(t_cs, style_map, weight: float = 1.0):
    """losses.py:84-87: earth_movers(hist(t_cs), hist(style_map)).mean(), differentiable in both
    arguments as the reference (train.py:261 passes data as style_map). `weight` fuses the caller's
    scale (train.py: 1e-5)."""
    x, y = _dev(t_cs, "t_cs"), _dev(style_map, "style_map")
    if x.shape[0] != y.shape[0]:
        raise Fn.HipOpError(f"hist loss: batch mismatch {tuple(x.shape)} vs {tuple(y.shape)}")
    return _two_sided(lambda a, b: _ops.hist_loss(a, b, float(weight))[0], x, y)


def out_of_range_loss(img, weight: float = 1e8):
    """train.py:259: compute_content_loss(img, torch.clip(img.detach(), 0.0, 1.0)) * 1e8."""
    return _ops.range_loss(_dev(img, "x"), float(weight))


def pixel_mse_loss(out, target, weight: float = 100.0):
    """train.py:268: ((target.detach() - out) ** 2).mean() * 100."""
    return _ops.sqdiff_mean(*_pair(out, target.detach(), "sqdiff"), float(weight))
