"""Drop-in for the reference losses.py (gram_matrix, compute_content_loss, compute_style_loss,
tv_loss). HIP kernels for these land with the training step."""
from __future__ import annotations

__all__ = ["gram_matrix", "compute_content_loss", "compute_style_loss", "tv_loss"]


def _pending(name):
    def f(*args, **kwargs):
        raise NotImplementedError(f"{name}: HIP kernel not implemented yet (SURVEY.md §8a A10-A13)")
    f.__name__ = name
    return f


gram_matrix = _pending("gram_matrix")
compute_content_loss = _pending("compute_content_loss")
compute_style_loss = _pending("compute_style_loss")
tv_loss = _pending("tv_loss")
