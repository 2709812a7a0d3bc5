"""Drop-in for the reference losses.py: gram_matrix, compute_content_loss, compute_style_loss,
tv_loss. Forward and backward are HIP kernels (functional.py).

The soft-histogram / Earth-Mover loss (losses.py:8-87, `compute_hist_loss`) is off the
north-star path (SURVEY.md §8f "next") and raises here.
"""
from __future__ import annotations

from . import functional as Fn

__all__ = ["gram_matrix", "compute_content_loss", "compute_style_loss", "tv_loss", "compute_hist_loss",
           "content_mvn_loss", "style_loss_weighted"]


def gram_matrix(tensor):
    """losses.py:105-109: bmm(F, F^T) / (C*H*W), F = tensor.view(B, C, H*W)."""
    return Fn.GramFn.apply(tensor)


def compute_content_loss(inp, tgt):
    """losses.py:124-126: F.huber_loss(inp, tgt) (delta 1, mean)."""
    return Fn.HuberFn.apply(inp, tgt)


def compute_style_loss(t_cs_map, style_map):
    """losses.py:128-139: 1.25*huber(mean) + 1.25*huber(std) + 10*huber(gram). The target is
    treated as a constant (train.py:233 always passes style_map[i].detach())."""
    return Fn.StyleLossFn.apply(t_cs_map, style_map.detach(), 1.0)


def tv_loss(img):
    """losses.py:90-103: sum of squared horizontal and vertical neighbour differences."""
    return Fn.TVLossFn.apply(img)


def content_mvn_loss(inp, tgt, weight: float = 1.0):
    """weight * compute_content_loss(mean_variance_norm(inp), mean_variance_norm(tgt.detach()))
    in one fused kernel (train.py:223-227, 258, 277)."""
    return Fn.MVNHuberFn.apply(inp, tgt.detach(), float(weight))


def style_loss_weighted(t_cs_map, style_map, weight: float = 1.0):
    """weight * compute_style_loss(t_cs_map, style_map.detach()) (train.py:230-245, 271)."""
    return Fn.StyleLossFn.apply(t_cs_map, style_map.detach(), float(weight))


def compute_hist_loss(t_cs, style_map):
    raise NotImplementedError("compute_hist_loss (losses.py:84-87) is off the AdaIN hot path "
                              "(SURVEY.md §8f rank 2); not implemented on HIP yet")
