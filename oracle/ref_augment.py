"""CPU oracle for the augmentation data path (SURVEY.md §8f "next" #3). TEST INFRASTRUCTURE ONLY
(tests/, bench scripts); the product path (arbitrarystyletransfer_amd.data_loader) never imports it.

The reference's get_transform (data_loader.py:110-135) runs torchvision transforms on tensors
(ToTensor is its first step). torchvision is not installed in this image, so its tensor kernels
are restated here with stock torch CPU ops, following torchvision's functional_tensor code:
rgb_to_grayscale, _blend, adjust_{brightness,contrast,saturation,hue} (_rgb2hsv / _hsv2rgb),
resize (= F.interpolate(mode="bilinear", antialias=True), torchvision >= 0.17's tensor default),
gaussian_blur (_get_gaussian_kernel1d, reflect padding, depthwise conv2d). Parity against
torchvision itself is therefore unpinned (no fixture of its outputs exists in the reference);
the geometric ops (rot90, flips) are exact torch ops.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def to_tensor(u8_hwc: torch.Tensor) -> torch.Tensor:
    """transforms.ToTensor on an RGB uint8 HWC array: fp32 CHW / 255."""
    return u8_hwc.permute(2, 0, 1).contiguous().to(torch.float32).div(255)


def rgb_to_grayscale(img: torch.Tensor, num_output_channels: int = 1) -> torch.Tensor:
    r, g, b = img.unbind(dim=-3)
    l_img = (0.2989 * r + 0.587 * g + 0.114 * b).to(img.dtype).unsqueeze(dim=-3)
    return l_img.expand(img.shape) if num_output_channels == 3 else l_img


def _blend(img1, img2, ratio):
    return (ratio * img1 + (1.0 - ratio) * img2).clamp(0, 1.0).to(img1.dtype)


def adjust_brightness(img, f):
    return _blend(img, torch.zeros_like(img), f)


def adjust_contrast(img, f):
    mean = torch.mean(rgb_to_grayscale(img).to(torch.float32), dim=(-3, -2, -1), keepdim=True)
    return _blend(img, mean, f)


def adjust_saturation(img, f):
    return _blend(img, rgb_to_grayscale(img), f)


def _rgb2hsv(img):
    r, g, b = img.unbind(dim=-3)
    maxc = torch.max(img, dim=-3).values
    minc = torch.min(img, dim=-3).values
    eqc = maxc == minc
    cr = maxc - minc
    ones = torch.ones_like(maxc)
    s = cr / torch.where(eqc, ones, maxc)
    cr_divisor = torch.where(eqc, ones, cr)
    rc = (maxc - r) / cr_divisor
    gc = (maxc - g) / cr_divisor
    bc = (maxc - b) / cr_divisor
    hr = (maxc == r) * (bc - gc)
    hg = ((maxc == g) & (maxc != r)) * (2.0 + rc - bc)
    hb = ((maxc != g) & (maxc != r)) * (4.0 + gc - rc)
    h = hr + hg + hb
    h = torch.fmod((h / 6.0 + 1.0), 1.0)
    return torch.stack((h, s, maxc), dim=-3)


def _hsv2rgb(img):
    h, s, v = img.unbind(dim=-3)
    i = torch.floor(h * 6.0)
    f = (h * 6.0) - i
    i = i.to(dtype=torch.int32)
    p = torch.clamp((v * (1.0 - s)), 0.0, 1.0)
    q = torch.clamp((v * (1.0 - s * f)), 0.0, 1.0)
    t = torch.clamp((v * (1.0 - s * (1.0 - f))), 0.0, 1.0)
    i = i % 6
    mask = i.unsqueeze(dim=-3) == torch.arange(6, device=i.device).view(-1, 1, 1)
    a1 = torch.stack((v, q, p, p, t, v), dim=-3)
    a2 = torch.stack((t, v, v, q, p, p), dim=-3)
    a3 = torch.stack((p, p, t, v, v, q), dim=-3)
    a4 = torch.stack((a1, a2, a3), dim=-4)
    return torch.einsum("...ijk, ...xijk -> ...xjk", mask.to(dtype=img.dtype), a4)


def adjust_hue(img, hue_factor):
    hsv = _rgb2hsv(img)
    h, s, v = hsv.unbind(dim=-3)
    h = (h + hue_factor) % 1.0
    return _hsv2rgb(torch.stack((h, s, v), dim=-3))


def resize(img, size):
    """transforms.Resize((h, w)) on a float tensor (antialiased bilinear)."""
    return F.interpolate(img.unsqueeze(0), size=list(size), mode="bilinear", align_corners=False,
                         antialias=True).squeeze(0)


def resized_crop(img, top, left, height, width, size):
    return resize(img[..., top:top + height, left:left + width], size)


def gaussian_kernel1d(kernel_size: int, sigma: float) -> torch.Tensor:
    ksize_half = (kernel_size - 1) * 0.5
    x = torch.linspace(-ksize_half, ksize_half, steps=kernel_size)
    pdf = torch.exp(-0.5 * (x / sigma).pow(2))
    return pdf / pdf.sum()


def gaussian_blur(img, kernel_size: int, sigma: float):
    k1 = gaussian_kernel1d(kernel_size, sigma).to(img.dtype)
    k2 = torch.mm(k1[:, None], k1[None, :])
    c = img.shape[-3]
    kernel = k2.expand(c, 1, kernel_size, kernel_size)
    pad = kernel_size // 2
    x = F.pad(img.unsqueeze(0), [pad, pad, pad, pad], mode="reflect")
    return F.conv2d(x, kernel, groups=c).squeeze(0)
