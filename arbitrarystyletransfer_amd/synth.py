"""Deterministic synthetic weights and inputs (the "live-init" recipe of SURVEY.md §8c).

No pretrained weights are reachable offline (the reference downloads ImageNet VGG19 at
models.py:192), and PyTorch-default inits give dead relu4_1 channels, so every
test, fixture and benchmark uses this counter-based generator. It is pure integer/float64 numpy,
so any language can regenerate the same float32 tensors bit for bit; the golden fixtures pin it
with per-layer checksums (tests/golden/).

    u_i(seed) = ((splitmix64(seed * 2**32 + i) >> 11) * 2**-53) * 2 - 1      in [-1, 1)

Conv weights: draw u for the whole [Cout, Cin/groups, k, k] tensor (seed = stream seed), remove
each filter's mean, rescale each filter to RMS sqrt(2 / fan_in); bias = 0.05 + 0.1 * U[0,1)
(seed + 1).  Images: u * 0.5 + 0.5 in [0, 1).
"""
from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser of (x + golden), vectorised over a uint64 array."""
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def uniform(seed: int, n: int) -> np.ndarray:
    """n float64 values in [-1, 1) from stream `seed`."""
    idx = np.arange(n, dtype=np.uint64) + np.uint64((seed & 0xFFFFFFFF) << 32)
    bits = splitmix64(idx) >> np.uint64(11)
    return bits.astype(np.float64) * (2.0 ** -53) * 2.0 - 1.0


def image(seed: int, shape) -> np.ndarray:
    """Synthetic image batch in [0, 1) (float32), e.g. shape (B, 3, H, W)."""
    n = int(np.prod(shape))
    return (uniform(seed, n) * 0.5 + 0.5).astype(np.float32).reshape(shape)


def conv_weight(seed: int, cout: int, cin_per_group: int, k: int) -> np.ndarray:
    """Zero-DC, RMS-normalised filter bank [cout, cin_per_group, k, k] (float32)."""
    fan_in = cin_per_group * k * k
    w = uniform(seed, cout * fan_in).reshape(cout, fan_in)
    w = w - w.mean(axis=1, keepdims=True)
    rms = np.sqrt((w * w).mean(axis=1, keepdims=True))
    w = w * (np.sqrt(2.0 / fan_in) / rms)
    return w.astype(np.float32).reshape(cout, cin_per_group, k, k)


def conv_bias(seed: int, cout: int) -> np.ndarray:
    return (0.05 + 0.1 * (uniform(seed, cout) * 0.5 + 0.5)).astype(np.float32)


def linear_weight(seed: int, out_f: int, in_f: int) -> np.ndarray:
    """SE Linear weight ~ U * 0.5 / sqrt(fan_in)."""
    return (uniform(seed, out_f * in_f) * 0.5 / np.sqrt(in_f)).astype(np.float32).reshape(out_f, in_f)


def linear_bias(seed: int, out_f: int) -> np.ndarray:
    """SE Linear bias in [0.4, 0.6] so the Hardtanh(0,1) gate sits near 0.5."""
    return (0.5 + 0.1 * uniform(seed, out_f)).astype(np.float32)


def bn_params(seed: int, c: int):
    """(gamma, beta, running_mean, running_var) for an eval-mode BatchNorm2d."""
    u = uniform(seed, 4 * c).reshape(4, c)
    gamma = 1.0 + 0.2 * u[0]
    beta = 0.1 * u[1]
    mean = 0.1 * u[2]
    var = 1.0 + 0.5 * u[3]
    return tuple(a.astype(np.float32) for a in (gamma, beta, mean, var))


def layer_seed(model_seed: int, layer_index: int) -> int:
    """Stream seed of parameter tensor `layer_index` of a model (two streams per layer)."""
    return model_seed * 1000 + 2 * layer_index


# --- VGG geometry (torchvision VGG19 "cfg E", restated; the reference imports it at models.py:192) ---

VGG19_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M",
             512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]


def vgg19_conv_shapes():
    """[(cin, cout)] of the 16 VGG19 convs, in order (conv_1 .. conv_16)."""
    shapes, cin = [], 3
    for v in VGG19_CFG:
        if v == "M":
            continue
        shapes.append((cin, v))
        cin = v
    return shapes


# The mirrored decoder spec at models.py:598-628: (cin, cout, upsample_before) per 3x3 conv.
VGG_DECODER_SPEC = [
    (512, 256, False),
    (256, 256, True),
    (256, 256, False),
    (256, 256, False),
    (256, 128, False),
    (128, 128, True),
    (128, 64, False),
    (64, 64, True),
    (64, 3, False),
]


def vgg_encoder_weights(model_seed: int = 1, n_convs: int = 16):
    """List of (weight, bias) for VGG19 conv_1..conv_n (live init)."""
    out = []
    for i, (cin, cout) in enumerate(vgg19_conv_shapes()[:n_convs]):
        s = layer_seed(model_seed, i)
        out.append((conv_weight(s, cout, cin, 3), conv_bias(s + 1, cout)))
    return out


def vgg_decoder_weights(model_seed: int = 2):
    out = []
    for i, (cin, cout, _) in enumerate(VGG_DECODER_SPEC):
        s = layer_seed(model_seed, i)
        out.append((conv_weight(s, cout, cin, 3), conv_bias(s + 1, cout)))
    return out


def live_init_(module, model_seed: int):
    """Apply the live-init recipe to every Conv2d / BatchNorm2d / Linear of `module`, in
    `named_modules()` order (leaf i uses streams layer_seed(model_seed, i) and +1).

    Works on the reference's MobileNet modules (mobilenetv2.py:95-181, models.py:140-338) and on
    this package's mirrors alike, because both have the same module tree. Returns `module`."""
    import torch
    import torch.nn as nn

    i = 0
    with torch.no_grad():
        for _, m in module.named_modules():
            s = layer_seed(model_seed, i)
            if isinstance(m, nn.Conv2d):
                kh, kw = m.kernel_size
                assert kh == kw
                w = conv_weight(s, m.out_channels, m.in_channels // m.groups, kh)
                m.weight.copy_(torch.from_numpy(w))
                if m.bias is not None:
                    m.bias.copy_(torch.from_numpy(conv_bias(s + 1, m.out_channels)))
            elif isinstance(m, nn.BatchNorm2d):
                g, b, mu, var = bn_params(s, m.num_features)
                m.weight.copy_(torch.from_numpy(g))
                m.bias.copy_(torch.from_numpy(b))
                m.running_mean.copy_(torch.from_numpy(mu))
                m.running_var.copy_(torch.from_numpy(var))
            elif isinstance(m, nn.Linear):
                m.weight.copy_(torch.from_numpy(linear_weight(s, m.out_features, m.in_features)))
                m.bias.copy_(torch.from_numpy(linear_bias(s + 1, m.out_features)))
            else:
                continue
            i += 1
    return module


def checksum(a: np.ndarray):
    """Order-independent fingerprint used by the fixtures to pin this generator."""
    a64 = np.asarray(a, dtype=np.float64).ravel()
    return np.array([a64.sum(), np.abs(a64).sum(), (a64 * a64).sum(),
                     a64[0], a64[len(a64) // 2], a64[-1]], dtype=np.float64)
