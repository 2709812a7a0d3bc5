"""Drop-in for the reference models.py: the same module names, constructor/forward signatures and
state-dict layouts, running on the HIP kernels of libast_hip.so.

`from arbitrarystyletransfer_amd.models import *` gives what `from models import *` gives the
reference callers (train.py:15-16): torch, nn, F, every conf name, the loss functions,
channel_stats / calc_mean_std / mean_variance_norm and the model classes.

Hot path: PretrainedEncoder(['relu_9']) -> AdaIN -> VGGDecoder, composed by
AdaINStyleTransfer. Tensors must live on a HIP device; there is no CPU fallback.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F  # noqa: F401  (re-exported like the reference)

from . import functional as Fn
from . import ops, synth
from .conf import *  # noqa: F401,F403
from .conf import device  # noqa: F401
from .losses import *  # noqa: F401,F403
from .model_util import channel_stats

IMNET_MEAN = (0.485, 0.456, 0.406)   # models.py:189
IMNET_STD = (0.229, 0.224, 0.225)    # models.py:190


class AdaIN(nn.Module):
    """AdaIN.forward, models.py:37-51, as one HIP launch (stats of both maps + normalise-affine).

    The reference unpacks channel_stats' (mean, std) as `style_std, style_mean` (models.py:44), so
    it computes (c - mu_c)/sigma_c * mu_s + sigma_s. That is the default here, for
    parity; `canonical=True` gives Huang & Belongie's (c - mu_c)/sigma_c * sigma_s + mu_s.
    `alpha` (default 1.0) fuses the blend of models.py:471: alpha * t + (1 - alpha) * content.
    """

    def __init__(self, canonical: bool = False):
        super().__init__()
        self.canonical = canonical

    def forward(self, content_map, style_map, alpha: float = 1.0):
        if torch.is_grad_enabled() and (content_map.requires_grad or style_map.requires_grad):
            return Fn.AdaINFn.apply(content_map, style_map, float(alpha), not self.canonical)
        return ops.adain(content_map, style_map, alpha=alpha, swap_style_stats=not self.canonical)


def calc_mean_std(feat, eps=1e-5):
    """models.py:54-62: per-(n,c) mean and sqrt(unbiased var + eps)."""
    if feat.dim() != 4:
        raise AssertionError("calc_mean_std expects a 4-D tensor")  # models.py:57
    return Fn.channel_stats(feat, unbiased=True, eps=eps)


def mean_variance_norm(feat):
    """models.py:64-68."""
    return Fn.mean_variance_norm(feat)


def _needs_grad(x, module):
    return torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in module.parameters()))


class Normalization(nn.Module):
    """models.py:120-131. Mean/std are non-persistent buffers: the reference keeps them as plain
    tensors, so they never appear in its state dict."""

    def __init__(self, mean, std):
        super().__init__()
        self.register_buffer("mean", torch.as_tensor(mean, dtype=torch.float32).view(-1, 1, 1), persistent=False)
        self.register_buffer("std", torch.as_tensor(std, dtype=torch.float32).view(-1, 1, 1), persistent=False)

    def forward(self, img):
        # Off the hot path: PretrainedEncoder fuses this into conv_1's gather.
        return (img - self.mean) / self.std


# --------------------------------------------------------------------------------------------
# VGG19 encoder / loss network
# --------------------------------------------------------------------------------------------

class _Named:
    @staticmethod
    def name(m: nn.Module, n: str) -> nn.Module:
        m.name = n
        return m


class _PackedConvCache:
    """Packed-weight copies of Conv2d modules, refreshed when the parameter changes."""

    def __init__(self):
        self._cache = {}

    def get(self, conv: nn.Conv2d) -> torch.Tensor:
        w = conv.weight
        key = id(conv)
        stamp = (w.data_ptr(), w._version, w.device, ops.WEIGHTS_EPOCH[0])
        hit = self._cache.get(key)
        if hit is not None and hit[0] == stamp:
            return hit[1]
        packed = ops.pack_conv3x3(w.detach())
        self._cache[key] = (stamp, packed)
        return packed


class PretrainedEncoder(nn.Module):
    """PretrainedEncoder, models.py:186-240: ImageNet normalisation + VGG19 `features` with layers
    named conv_i / relu_i / pool_i (models.py:199-224), returning the requested layers in network
    order and stopping once all are collected (models.py:235-238).

    `_vgg_layers` keeps the reference's ModuleList indices (Normalization at 0, torchvision
    features.N at N+1), so state dicts interchange. Weights: the reference downloads ImageNet
    VGG19 (models.py:192), which is unavailable offline; `weights="live"` (default) uses the
    deterministic live-init recipe (synth.py, seed `seed`), `weights=None` leaves PyTorch's
    default init; load real weights with load_state_dict / load_torchvision_features.

    HIP execution: each conv is one fused launch (conv_1 also applies the normalisation); ReLU and
    2x2 max-pool run in the conv epilogue; the pre-ReLU conv_i taps are dual-stored.
    """

    def __init__(self, content_layers=("conv_1", "conv_3", "conv_5", "conv_9", "conv_13", "relu_15"),
                 weights="live", seed: int = 1):
        super().__init__()
        self._content_layers = set(content_layers)
        norm = _Named.name(Normalization(IMNET_MEAN, IMNET_STD), "norm")
        layers = [norm]
        i, cin = 0, 3
        for v in synth.VGG19_CFG:
            if v == "M":
                layers.append(_Named.name(nn.MaxPool2d(kernel_size=2, stride=2), f"pool_{i}"))
            else:
                i += 1
                layers.append(_Named.name(nn.Conv2d(cin, v, kernel_size=3, padding=1), f"conv_{i}"))
                layers.append(_Named.name(nn.ReLU(inplace=False), f"relu_{i}"))
                cin = v
        self._vgg_layers = nn.ModuleList(layers)
        if weights == "live":
            self.load_live_init(seed)
        self._packed = _PackedConvCache()

    def convs(self):
        return [m for m in self._vgg_layers if isinstance(m, nn.Conv2d)]

    @torch.no_grad()
    def load_live_init(self, seed: int = 1):
        for conv, (w, b) in zip(self.convs(), synth.vgg_encoder_weights(seed)):
            conv.weight.copy_(torch.from_numpy(w))
            conv.bias.copy_(torch.from_numpy(b))

    @torch.no_grad()
    def load_torchvision_features(self, state_dict):
        """Load a torchvision vgg19().features state dict (keys 'N.weight' / 'N.bias')."""
        mapped = {f"_vgg_layers.{int(k.split('.')[0]) + 1}.{k.split('.', 1)[1]}": v for k, v in state_dict.items()}
        self.load_state_dict(mapped)

    def _plan(self):
        """[(conv_index, conv, want_pre, want_act, want_pool, [names collected in order])]."""
        wanted = self._content_layers
        got = set()
        plan = []
        mods = list(self._vgg_layers)
        k = 1
        while k < len(mods) and len(got) < len(wanted):
            conv = mods[k]
            idx = int(conv.name.split("_")[1])
            pool_follows = k + 2 < len(mods) and isinstance(mods[k + 2], nn.MaxPool2d)
            names = [conv.name, f"relu_{idx}"] + ([f"pool_{idx}"] if pool_follows else [])
            collect = [nm for nm in names if nm in wanted]
            got.update(collect)
            more = len(got) < len(wanted)
            want_pre = conv.name in wanted
            want_act = f"relu_{idx}" in wanted or (more and not pool_follows)
            want_pool = pool_follows and (f"pool_{idx}" in wanted or more)
            plan.append((idx, conv, want_pre, want_act, want_pool, collect))
            k += 3 if pool_follows else 2
        return plan

    def forward(self, x, x2=None):
        """Feature maps of the requested layers. `x2` (optional, same C/H/W): a second batch
        encoded in the same launches, outputs hold x's images then x2's."""
        norm = self._vgg_layers[0]
        if _needs_grad(x, self) or (x2 is not None and _needs_grad(x2, self)):
            if x2 is not None:
                return [torch.cat(p) for p in zip(self._forward_autograd(x), self._forward_autograd(x2))]
            return self._forward_autograd(x)
        outs = []
        cur, cur2 = x, x2
        for idx, conv, want_pre, want_act, want_pool, collect in self._plan():
            first = idx == 1
            pre, act, pool = ops.conv3x3(
                cur, self._packed.get(conv), conv.bias, conv.out_channels, pad_mode="zeros",
                in_mean=norm.mean.view(-1) if first else None, in_std=norm.std.view(-1) if first else None,
                want_pre=want_pre, want_act=want_act, want_pool=want_pool, x2=cur2)
            by_name = {conv.name: pre, f"relu_{idx}": act, f"pool_{idx}": pool}
            outs.extend(by_name[nm] for nm in collect)
            cur, cur2 = (pool if want_pool else act), None
        return outs

    def _forward_autograd(self, x):
        """Same walk through EncoderConvFn (HIP forward + HIP backward; the pre-ReLU output is
        always kept for the ReLU / max-pool backward)."""
        norm = self._vgg_layers[0]
        outs = []
        cur = x
        for idx, conv, want_pre, want_act, want_pool, collect in self._plan():
            first = idx == 1
            pre, act, pool = Fn.EncoderConvFn.apply(
                cur, conv.weight, conv.bias, self._packed.get(conv), want_act, want_pool,
                norm.mean.view(-1) if first else None, norm.std.view(-1) if first else None)
            by_name = {conv.name: pre, f"relu_{idx}": act, f"pool_{idx}": pool}
            outs.extend(by_name[nm] for nm in collect)
            cur = pool if want_pool else act
        return outs


# --------------------------------------------------------------------------------------------
# Mirrored VGG decoder (models.py:598-628)
# --------------------------------------------------------------------------------------------

class VGGDecoder(nn.Sequential):
    """The mirrored decoder spec at models.py:598-628 (a commented nn.Sequential in the
    reference), with the same Sequential indices so its state dict interchanges. Each
    [Upsample] + ReflectionPad + Conv + [ReLU] group is one fused HIP launch."""

    def __init__(self, weights="live", seed: int = 2):
        layers = []
        for cin, cout, up in synth.VGG_DECODER_SPEC:
            if up:
                layers.append(nn.Upsample(scale_factor=2, mode="nearest"))
            layers += [nn.ReflectionPad2d((1, 1, 1, 1)), nn.Conv2d(cin, cout, (3, 3))]
            if cout != 3:
                layers.append(nn.ReLU())
        super().__init__(*layers)
        self._groups = []
        up = False
        mods = list(self)
        for k, m in enumerate(mods):
            if isinstance(m, nn.Upsample):
                up = True
            elif isinstance(m, nn.Conv2d):
                relu = k + 1 < len(mods) and isinstance(mods[k + 1], nn.ReLU)
                self._groups.append((m, up, relu))
                up = False
        if weights == "live":
            self.load_live_init(seed)
        object.__setattr__(self, "_packed", _PackedConvCache())

    def convs(self):
        return [g[0] for g in self._groups]

    @torch.no_grad()
    def load_live_init(self, seed: int = 2):
        for conv, (w, b) in zip(self.convs(), synth.vgg_decoder_weights(seed)):
            conv.weight.copy_(torch.from_numpy(w))
            conv.bias.copy_(torch.from_numpy(b))

    def forward(self, x):
        if _needs_grad(x, self):
            for conv, up, relu in self._groups:
                x = Fn.DecoderConvFn.apply(x, conv.weight, conv.bias, self._packed.get(conv), 2 if up else 1, relu)
            return x
        for conv, up, relu in self._groups:
            pre, act, _ = ops.conv3x3(x, self._packed.get(conv), conv.bias, conv.out_channels,
                                      upsample=2 if up else 1, pad_mode="reflect",
                                      want_pre=not relu, want_act=relu)
            x = act if relu else pre
        return x


class AdaINStyleTransfer(nn.Module):
    """encoder (VGG19 to relu4_1) -> AdaIN -> alpha blend -> mirrored decoder.

    forward(content_img, style_img, alpha=1.0) -> stylised image [B, 3, H, W]. Content and
    style batches of the same shape are encoded in the same launches.
    """

    def __init__(self, canonical: bool = False, enc_seed: int = 1, dec_seed: int = 2, weights="live"):
        super().__init__()
        self.encoder = PretrainedEncoder(content_layers=["relu_9"], weights=weights, seed=enc_seed)
        self.adain = AdaIN(canonical=canonical)
        self.decoder = VGGDecoder(weights=weights, seed=dec_seed)

    def encode_pair(self, content_img, style_img):
        if content_img.shape[1:] == style_img.shape[1:]:
            f = self.encoder(content_img, style_img)[0]
            b = content_img.shape[0]
            return f[:b], f[b:]
        return self.encoder(content_img)[0], self.encoder(style_img)[0]

    def forward(self, content_img, style_img, alpha: float = 1.0):
        f_c, f_s = self.encode_pair(content_img, style_img)
        t = self.adain(f_c, f_s, alpha=alpha)
        return self.decoder(t)
