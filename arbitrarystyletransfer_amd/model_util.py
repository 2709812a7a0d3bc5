"""Drop-in for the reference model_util.py (hot-path part).

channel_stats (model_util.py:3-8) runs on the HIP channel-statistics kernel. The RGB<->Lab
colour helpers (model_util.py:11-140) are off the hot path (out of scope).
"""
from . import functional


def channel_stats(img):
    """Per-(n,c) spatial mean and unbiased std (no eps), keepdim: model_util.py:3-8."""
    return functional.channel_stats(img, unbiased=True, eps=0.0)
