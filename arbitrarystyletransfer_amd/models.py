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
from . import mbtrain, ops, synth
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
        if _compiling():   # torch.compile: the registered op (fake impl + autograd), no graph break
            return torch.ops.ast_hip.adain_map(content_map, style_map, float(alpha), not self.canonical)
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


class AdaAttN(nn.Module):
    """AdaAttN, models.py:70-115: attention-weighted style mean/std (SURVEY.md §8f "next" #1).

    Same module tree as the reference (W_q/W_k/W_v 1x1 convs without bias, att_act, std_act and
    the three parameter-free InstanceNorm2d), so state dicts load unchanged. forward runs
    ops.adaattn: the Nq x Nk attention matrix is never materialised (one fused HIP kernel). Under
    autograd (fp32, training the reference's AST, train.py:287-300) the backward recomputes the
    attention on the MFMA GEMMs (attention.AdaAttNFn) and yields gradients for W_q, W_k, W_v and
    both inputs.
    """

    def __init__(self, inp_size):
        super().__init__()
        self.W_q = nn.Conv2d(inp_size, inp_size, 1, 1, 0, bias=False)
        self.W_k = nn.Conv2d(inp_size, inp_size, 1, 1, 0, bias=False)
        self.W_v = nn.Conv2d(inp_size, inp_size, 1, 1, 0, bias=False)
        self.att_act = nn.Softmax(dim=-1)
        self.std_act = nn.ReLU(True)
        self.inst_norm_1 = nn.InstanceNorm2d(inp_size)
        self.inst_norm_2 = nn.InstanceNorm2d(inp_size)
        self.inst_norm = nn.InstanceNorm2d(inp_size)
        self.inp_size = inp_size

    def forward(self, content_map, style_map):
        if content_map.shape[1] != self.inp_size:
            raise ops.HipOpError(f"expected {self.inp_size} channels, got {content_map.shape[1]}")
        if torch.is_grad_enabled() and (content_map.requires_grad or style_map.requires_grad
                                        or any(p.requires_grad for p in self.parameters())):
            from . import attention
            return attention.adaattn(self, content_map, style_map)
        return ops.adaattn(content_map, style_map, self.W_q.weight, self.W_k.weight, self.W_v.weight)


def _compiling() -> bool:
    """Under torch.compile / dynamo tracing the modules call torch.ops.ast_hip.* (library.py: the
    same C-ABI kernels behind registered custom ops with fake implementations) and pack weights
    with the ast_hip::conv3x3_pack op instead of the data_ptr-keyed caches, which dynamo cannot
    trace. Eager calls keep the direct C-ABI launches (no dispatcher overhead per launch)."""
    return torch.compiler.is_compiling()


def _ops():
    from . import library  # noqa: F401  (registers the ast_hip::* custom ops)
    return torch.ops.ast_hip


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
        stamp = (w.data_ptr(), w._version, w.device, ops.weight_epoch(w))
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
        if _compiling():
            return self._forward_ops(x, x2)
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

    def _forward_ops(self, x, x2=None):
        """The same walk through torch.ops.ast_hip.conv3x3 (torch.compile path; with autograd its
        registered backward runs the same HIP dgrad / wgrad kernels)."""
        A = _ops()
        norm = self._vgg_layers[0]
        outs = []
        cur, cur2 = x, x2
        grad = x2 is None and _needs_grad(x, self)
        for idx, conv, want_pre, want_act, want_pool, collect in self._plan():
            first = idx == 1
            pre, act, pool = A.conv3x3(cur, conv.weight, A.conv3x3_pack(conv.weight.detach()), conv.bias, 1, 0,
                                       norm.mean.view(-1) if first else None, norm.std.view(-1) if first else None,
                                       want_pre or grad, want_act, want_pool, cur2)
            by_name = {conv.name: pre, f"relu_{idx}": act, f"pool_{idx}": pool}
            outs.extend(by_name[nm] for nm in collect)
            cur, cur2 = (pool if want_pool else act), None
        return outs

    def prepack(self):
        """Build the forward and input-gradient weight packs of every conv this network runs, ahead
        of a hipGraph capture (train.StepGraph): the loss network is frozen, so its packs are made
        once, outside the graph, instead of being rebuilt by every replay."""
        norm = self._vgg_layers[0]
        for idx, conv, *_ in self._plan():
            self._packed.get(conv)
            Fn._TF.get(conv.weight, norm.std.view(-1) if idx == 1 else None)

    def _forward_autograd(self, x):
        """Same walk through EncoderConvFn (HIP forward + HIP backward; the pre-ReLU output is
        always kept for the ReLU / max-pool backward); frozen weights: one LossNetFn node for the
        whole walk (cross-layer fused backward)."""
        if not any(p.requires_grad for p in self.parameters()):
            return list(Fn.LossNetFn.apply(self, x))
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
        if _compiling():
            A = _ops()
            for conv, up, relu in self._groups:
                pre, act, _ = A.conv3x3(x, conv.weight, A.conv3x3_pack(conv.weight.detach()), conv.bias,
                                        2 if up else 1, 1, None, None, not relu, relu, False, None)
                x = act if relu else pre
            return x
        if _needs_grad(x, self):
            # each ReLU output feeds only the next conv: its ReLU backward runs in that conv's
            # input-gradient epilogue (mask_input), and the layer itself passes its gradient through
            g = self._groups
            for k, (conv, up, relu) in enumerate(g):
                x = Fn.DecoderConvFn.apply(x, conv.weight, conv.bias, self._packed.get(conv), 2 if up else 1, relu,
                                           k > 0 and g[k - 1][2], relu and k + 1 < len(g))
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

    # -- one style, many contents: the style owner encodes the style once and
    #    broadcasts its relu4_1 statistics (dp.broadcast_style_stats, 2*512 floats) --------------
    def style_statistics(self, style_img):
        """(mean, std) of the style's relu4_1 features, each [N_style, 512]."""
        f_s = self.encoder(style_img)[0]
        m, s = channel_stats(f_s)
        return m.flatten(1), s.flatten(1)

    def stylize_with_stats(self, content_img, style_mean, style_std, alpha: float = 1.0):
        """Stylise a content batch with given style statistics ([512] shared, or [N, 512])."""
        if torch.is_grad_enabled() and (content_img.requires_grad or any(p.requires_grad for p in self.parameters())):
            raise NotImplementedError("stylize_with_stats is inference-only; run it under torch.no_grad()")
        f_c = self.encoder(content_img)[0]
        t = ops.adain_stats(f_c, style_mean, style_std, alpha=alpha, swap_style_stats=not self.adain.canonical)
        return self.decoder(t)


# ------------------------------------------------------------------------------------------------
# MobileNet-style variant: Encoder -> per-layer AdaIN -> ada_out ->
# Decoder. Blocks are the DepthWiseConv/conv_3x3_bn mirrors of mobilenetv2.py (HIP forwards).
# ------------------------------------------------------------------------------------------------
from .mobilenetv2 import DTYPE_CODE, DepthWiseConv, SELayer, _make_divisible, act_dtype, check_inference  # noqa: E402,F401
from .mobilenetv2 import _trace_io  # noqa: E402
from .mobilenetv2 import conv_3x3_bn  # noqa: E402,F401
from ._lib import HipOpError, check, lib, ptr, stream_ptr  # noqa: E402


class Encoder(nn.Module):
    """models.py:140-184: conv_3x3_bn + 14 DepthWiseConv blocks from conf.enc_conv_shapes; returns
    the outputs of the blocks listed in out_layers. BatchNorm uses running statistics (eval)."""

    def __init__(self, exporting=False, use_inst_norm=False):
        super().__init__()
        blocks = [conv_3x3_bn(enc_conv_shapes[0][0], enc_conv_shapes[0][1], enc_conv_shapes[0][2])]
        for in_ch, out_ch, stride, kernel_size, expand_ratio in enc_conv_shapes[1:-1]:
            blocks.append(DepthWiseConv(in_ch, out_ch, stride, expand_ratio, use_norm=True, kernel_size=kernel_size))
        # models.py:153: the last block reuses the loop's final (in, out, stride) with EXPAND_RATIO
        blocks.append(DepthWiseConv(in_ch, out_ch, stride, EXPAND_RATIO, use_norm=True))
        self.mob_net = nn.ModuleList(blocks)

    def forward(self, x, out_layers=[], auto_enc=False):
        if auto_enc:
            for layer in self.mob_net:
                x = layer(x)
            return x
        outs = []
        last = max(out_layers) if len(out_layers) else -1   # later blocks cannot change the result
        if self.training and mbtrain.wants_training_path(self, x):
            last = len(self.mob_net) - 1   # train mode: every block runs (BatchNorm running statistics)
        for i, layer in enumerate(self.mob_net):
            if i > last:
                break
            x = layer(x)
            if i in out_layers:
                outs.append(x)
        return outs


class DecoderBlock(nn.Module):
    """models.py:242-272: DepthWiseConv (no BN), then optionally nearest Upsample x2 + ratio-1
    DepthWiseConv (the upsample is fused into that block's depthwise gather)."""

    def __init__(self, in_channels, out_channels, stride, kernel_size=3, upsample=False, expand_ratio=6):
        super().__init__()
        self._ref_pad = nn.ReflectionPad2d((1, 1, 1, 1))
        self._conv = DepthWiseConv(in_channels, out_channels, stride, expand_ratio, use_norm=False,
                                   kernel_size=kernel_size)
        self._should_upsample = upsample
        if self._should_upsample:
            self._ref_out = nn.ReflectionPad2d((1, 1, 1, 1))
            self._upsample_2 = DepthWiseConv(out_channels, out_channels, 1, 1, use_norm=False)
            self._upsample_3 = nn.Upsample(scale_factor=2, mode="nearest")

    def forward(self, x):
        x = self._conv(x)
        if self._should_upsample:
            x = self._upsample_2.run(x, None, up=2)   # training path: explicit upsample, then the block
        return x


class Decoder(nn.Module):
    """models.py:274-320: 14 DecoderBlocks from conf.decoder_conv_shapes (upsample where the
    channel count changes and i + 6 < 15, models.py:284), ReflectionPad + Conv(16->3, bias), and
    Hardtanh(0, 1) only when exporting. Output in the parameters' dtype."""

    def __init__(self, exporting=False):
        super().__init__()
        self.exporting = exporting
        blocks = []
        for i, conv_shape in enumerate(decoder_conv_shapes[:-1]):
            should_upsample = conv_shape[0] != conv_shape[1] and i + 6 < len(decoder_conv_shapes)
            blocks.append(DecoderBlock(conv_shape[0], conv_shape[1], conv_shape[2], upsample=should_upsample,
                                       expand_ratio=conv_shape[4], kernel_size=conv_shape[3]))
        self._decoder_blocks = nn.ModuleList(blocks)
        self._ref_out = nn.ReflectionPad2d((1, 1, 1, 1))
        self._img_out = nn.Conv2d(decoder_conv_shapes[-1][0], decoder_conv_shapes[-1][1], kernel_size=(3, 3))
        self.last_act = nn.Hardtanh(0.0, 1.0)

    def forward(self, x):
        for block in self._decoder_blocks:
            x = block(x)
        return self._image_conv(x)

    def _image_conv(self, x):
        conv = self._img_out
        if mbtrain.wants_training_path(self, x):
            y = Fn.DecoderConvFn.apply(x.float().contiguous(), conv.weight, conv.bias,
                                       ops.pack_conv3x3(conv.weight.detach().float()), 1, False)
            if self.exporting:
                raise NotImplementedError("Hardtanh output under autograd (exporting=True) is inference-only")
            return y
        check_inference(x, self)
        dt = act_dtype(self)
        if x.dtype != dt or x.device.type != "cuda" or x.dim() != 4 or x.shape[1] != conv.in_channels:
            raise HipOpError(f"decoder output conv expects ({conv.in_channels}-channel NCHW {dt} on HIP), "
                             f"got {tuple(x.shape)} {x.dtype} on {x.device}")
        x = x.contiguous()
        n, _, h, w = x.shape
        stamp = (dt, x.device, ops.weight_epoch(conv.weight), ops.weight_epoch(conv.bias), conv.weight._version,
                 conv.bias._version, conv.weight.data_ptr())
        if getattr(self, "_out_stamp", None) != stamp:
            self._w = conv.weight.detach().float().contiguous()
            self._b = conv.bias.detach().float().contiguous()
            self._out_stamp = stamp
        y = torch.empty((n, conv.out_channels, h, w), device=x.device, dtype=dt)
        nbytes = x.numel() * x.element_size() + y.numel() * y.element_size()
        _trace_io(nbytes)
        check(ops._timed("mb dense3x3 out", -nbytes, x.device, lambda: lib().ast_mb_conv3x3_dense(
            DTYPE_CODE[dt], DTYPE_CODE[dt], ptr(x), ptr(self._w), ptr(self._b), ptr(y), n, conv.in_channels,
            conv.out_channels, h, w, 2 if self.exporting else 0, stream_ptr(x.device))), "decoder output conv")
        return y


class AutoEncoder(nn.Module):
    """models.py:322-338: Encoder -> cat(layers 12, 14) -> ada_out -> Decoder."""

    def __init__(self):
        super().__init__()
        self.encoder = Encoder(use_inst_norm=True)
        self.ada_out = DepthWiseConv(enc_out_channels * 2, enc_out_channels, 1, EXPAND_RATIO, use_norm=False,
                                     use_identity=False)
        self.decoder = Decoder()

    def load_live_init(self, enc_seed: int = 5, dec_seed: int = 6, ada_seed: int = 7):
        synth.live_init_(self.encoder, enc_seed)
        synth.live_init_(self.decoder, dec_seed)
        synth.live_init_(self.ada_out, ada_seed)
        return self

    def forward(self, x):
        enc_x = self.encoder(x, out_layers=enc_out_layers)
        return self.decoder(self.ada_out(enc_x[0], enc_x[1]))


class AST(nn.Module):
    """The reference AST (models.py:393-582), MobileNet-variant encoder -> per-layer stylisation
    at enc_out_layers -> ada_out -> decoder.

    The reference class does not run (SyntaxError at models.py:459; ada_att_2 and
    ada_out are used by encode (models.py:557-565) but not defined). This keeps the constructor
    and forward signatures and return values (models.py:395,425,529-533) and the encode structure
    (models.py:535-566). `attention=False` (default, the north-star path) stylises each layer with
    AdaIN(content_i, style_i); `attention=True` uses the reference's own choice, AdaAttN modules
    `ada_att_1` / `ada_att_2` (models.py:407-408, 557-558), each over enc_out_channels.
    Train mode with autograd (ASTTrainer, train.py:146-300) runs the training kernels: the
    detached eval-mode encoding of encode(detach=True), AdaAttN / ada_out / decoder with backward,
    and the train-mode (batch statistics) content encoding feeding org_out, as models.py:425-476.
    """

    def __init__(self, style_layers=[4, 7, 10, 12, 16], content_layers=[4, 7, 10, 12, 16], exporting=False,
                 attention=False):
        super().__init__()
        self._style_layers = style_layers
        self._content_layers = content_layers
        self._exporting = exporting
        self._enc = Encoder(self._exporting)
        self._dec = Decoder(self._exporting)
        self._attention = attention
        if attention:
            self.ada_att_1 = AdaAttN(enc_out_channels)
            self.ada_att_2 = AdaAttN(enc_out_channels)
        else:
            self._adain = AdaIN()
        self.ada_out = DepthWiseConv(enc_out_channels * 2, enc_out_channels, 1, EXPAND_RATIO, use_norm=False,
                                     use_identity=False)

    def load_live_init(self, enc_seed: int = 5, dec_seed: int = 6, ada_seed: int = 7, att_seed: int = 8):
        synth.live_init_(self._enc, enc_seed)
        synth.live_init_(self._dec, dec_seed)
        synth.live_init_(self.ada_out, ada_seed)
        if self._attention:
            synth.live_init_(self.ada_att_1, att_seed)
            synth.live_init_(self.ada_att_2, att_seed + 1)
        return self

    def stylize_maps(self, content_maps, style_maps):
        """Per-layer stylisation of the enc_out_layers maps (models.py:557-558)."""
        if self._attention:
            return self.ada_att_1(content_maps[0], style_maps[0]), self.ada_att_2(content_maps[1], style_maps[1])
        for m in content_maps:     # AdaIN reads content + style and writes its output
            _trace_io(3 * m.numel() * m.element_size())
        return self._adain(content_maps[0], style_maps[0]), self._adain(content_maps[1], style_maps[1])

    def encode(self, content_img, style_img, detach=False, return_maps=False):
        """models.py:535-566. detach=True: the encoder runs in eval mode (running statistics) and its
        maps are detached (models.py:537-545), so it runs here without recording autograd."""
        if detach:
            was = self._enc.training
            self._enc.eval()
            with torch.no_grad():
                content_maps = self._enc(content_img, out_layers=enc_out_layers)
                style_maps = self._enc(style_img, out_layers=enc_out_layers)
            self._enc.train(was)
        else:
            content_maps = self._enc(content_img, out_layers=enc_out_layers)
            style_maps = self._enc(style_img, out_layers=enc_out_layers)
        st1, st2 = self.stylize_maps(content_maps, style_maps)
        stylized_map = self.ada_out(st1, st2)
        self._last_content_maps = content_maps
        if return_maps:
            return st1, st2, stylized_map
        return stylized_map

    def forward(self, content_img, style_img, alpha=1.0):
        """models.py:425-533: t_cs when exporting, else (t_cs, t_return, org_out).

        t_return = (stylized_map_1, stylized_map_2), the per-layer stylised maps: train.py:276-277
        pairs t[i] with the stylised image's encoding at each of enc_out_layers, and calc_mean_std
        asserts 4-D maps (models.py:57), so this is the reading of the unparsable models.py:459
         under which the reference's training loop runs."""
        if self._exporting:
            t = self.encode(content_img, style_img)
            self._last_content_maps = None
            return self._dec(t)
        st1, st2, t = self.encode(content_img, style_img, detach=True, return_maps=True)
        if self.training:
            # train mode: the content encoding for org_out uses batch statistics (and updates the
            # running ones), as the reference's second encoder call does (models.py:466-469)
            c = self._enc(content_img, out_layers=enc_out_layers)
        else:
            c = self._last_content_maps    # eval mode: the same maps encode() just computed
        self._last_content_maps = None
        content_map = self.ada_out(c[0], c[1])
        if alpha != 1.0:
            t = alpha * t + (1 - alpha) * content_map
        org_out = self._dec(content_map)
        t_cs = self._dec(t)
        return t_cs, (st1, st2), org_out
