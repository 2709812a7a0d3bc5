"""HIP kernels of the augmentation data path (csrc/augment.hip; SURVEY.md §8f "next" #3) on
[C, H, W] fp32 device images, with torchvision's tensor semantics (the reference applies its
transforms after ToTensor). Random parameters are drawn by the caller (data_loader.py)."""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from ._lib import HipOpError, check, lib, loss_accumulator, ptr, stream_ptr

COLOR_OPS = {"brightness": 0, "contrast": 1, "saturation": 2, "hue": 3, "grayscale": 4}


def _img(x: torch.Tensor, name: str = "img") -> torch.Tensor:
    if not isinstance(x, torch.Tensor):
        raise TypeError(f"{name} must be a tensor")
    if x.device.type != "cuda":
        raise HipOpError(f"{name} is on {x.device}; the augmentation kernels run on MI355X (HIP) devices only")
    if x.dim() != 3 or x.dtype != torch.float32:
        raise HipOpError(f"{name} must be a float32 [C, H, W] tensor, got {x.dtype} {tuple(x.shape)}")
    return x.contiguous()


def to_tensor(image, device) -> torch.Tensor:
    """transforms.ToTensor for an RGB image (PIL image or uint8 HWC array): the uint8 bytes are
    copied to the device (a quarter of the float bytes) and converted there."""
    arr = np.asarray(image)
    if arr.dtype != np.uint8 or arr.ndim != 3 or arr.shape[2] < 3:
        raise HipOpError(f"to_tensor expects an RGB uint8 HWC image, got {arr.dtype} {arr.shape}")
    h, w, cs = arr.shape
    src = torch.from_numpy(np.ascontiguousarray(arr)).to(device, non_blocking=True)
    out = torch.empty((3, h, w), device=device, dtype=torch.float32)
    check(lib().ast_aug_to_tensor(ptr(src), h, w, cs, ptr(out), stream_ptr(out.device)), "to_tensor")
    return out


def _remap(img, ho, wo, coef):
    img = _img(img)
    c, h, w = img.shape
    out = torch.empty((c, ho, wo), device=img.device, dtype=torch.float32)
    arr = (ctypes.c_int * 6)(*coef)
    check(lib().ast_aug_remap_f32(ptr(img), c, h, w, ptr(out), ho, wo, ctypes.cast(arr, ctypes.c_void_p),
                                  stream_ptr(img.device)), "remap")
    return out


def rot90(img, k: int):
    """torch.rot90(img, k, [1, 2]) for k in {1, -1} (data_loader.py:22)."""
    c, h, w = img.shape
    k %= 4
    if k == 1:
        return _remap(img, w, h, (0, 1, 0, -1, 0, w - 1))
    if k == 3:
        return _remap(img, w, h, (0, -1, h - 1, 1, 0, 0))
    if k == 2:
        return _remap(img, h, w, (-1, 0, h - 1, 0, -1, w - 1))
    return img


def hflip(img):
    c, h, w = img.shape
    return _remap(img, h, w, (1, 0, 0, 0, -1, w - 1))


def vflip(img):
    c, h, w = img.shape
    return _remap(img, h, w, (-1, 0, h - 1, 0, 1, 0))


def _color(img, op, factor=0.0, gsum=None):
    img = _img(img)
    if img.shape[0] != 3:
        raise HipOpError("colour adjustments need a 3-channel image")
    _, h, w = img.shape
    out = torch.empty_like(img)
    check(lib().ast_aug_color_f32(ptr(img), h, w, COLOR_OPS[op], float(factor), ptr(gsum), ptr(out),
                                  stream_ptr(img.device)), op)
    return out


def adjust_brightness(img, f):
    return _color(img, "brightness", f)


def adjust_contrast(img, f):
    img = _img(img)
    gsum = loss_accumulator(img.device)   # the sum lands in element 0 (fixed-order reduction)
    check(lib().ast_aug_gray_sum_f32(ptr(img), img.shape[1], img.shape[2], ptr(gsum), stream_ptr(img.device)),
          "gray_sum")
    return _color(img, "contrast", f, gsum)


def adjust_saturation(img, f):
    return _color(img, "saturation", f)


def adjust_hue(img, f):
    if not -0.5 <= f <= 0.5:
        raise ValueError(f"hue_factor ({f}) is not in [-0.5, 0.5].")
    return _color(img, "hue", f)


def rgb_to_grayscale3(img):
    return _color(img, "grayscale")


def resized_crop(img, top: int, left: int, height: int, width: int, size):
    """resize(img[:, top:top+height, left:left+width], size), antialiased bilinear."""
    img = _img(img)
    c, h, w = img.shape
    ho, wo = int(size[0]), int(size[1])
    out = torch.empty((c, ho, wo), device=img.device, dtype=torch.float32)
    tmp = torch.empty((lib().ast_aug_resize_workspace_floats(c, height, wo),), device=img.device,
                      dtype=torch.float32)
    check(lib().ast_aug_resize_f32(ptr(img), c, h, w, int(top), int(left), int(height), int(width), ptr(out), ho, wo,
                                   ptr(tmp), stream_ptr(img.device)), "resize")
    return out


def resize(img, size):
    """transforms.Resize((h, w)) on a tensor (antialias=True, torchvision >= 0.17 default)."""
    return resized_crop(img, 0, 0, img.shape[1], img.shape[2], size)


def gaussian_kernel1d(kernel_size: int, sigma: float):
    """torchvision's _get_gaussian_kernel1d, in fp32 on the host (k <= 15 taps)."""
    half = (kernel_size - 1) * 0.5
    x = torch.linspace(-half, half, steps=kernel_size)
    pdf = torch.exp(-0.5 * (x / sigma).pow(2))
    return (pdf / pdf.sum()).tolist()


def gaussian_blur(img, kernel_size: int, sigma: float):
    img = _img(img)
    c, h, w = img.shape
    taps = (ctypes.c_float * kernel_size)(*gaussian_kernel1d(kernel_size, sigma))
    out = torch.empty_like(img)
    tmp = torch.empty_like(img)
    check(lib().ast_aug_blur_f32(ptr(img), c, h, w, ctypes.cast(taps, ctypes.c_void_p), kernel_size, ptr(out),
                                 ptr(tmp), stream_ptr(img.device)), "gaussian_blur")
    return out
