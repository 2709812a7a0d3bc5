"""GPU parity for the on-device augmentation path (SURVEY.md §8f "next" #3; data_loader.py:110-135)
against oracle/ref_augment.py (torchvision's tensor formulas restated with torch CPU ops;
torchvision itself is absent, so parity against the library is unpinned).

Bars: geometric ops and ToTensor bit-exact; colour ops, resize and blur rel_inf <= 2e-5 (fp32
summation-order differences); the seeded end-to-end pipeline <= 1e-4.
"""
import random
import types

import numpy as np
import pytest
import torch

from arbitrarystyletransfer_amd import augment as A
from arbitrarystyletransfer_amd import data_loader as DL
from oracle import ref_augment as R

pytestmark = pytest.mark.gpu


def rel_inf(a, b):
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


def u8_image(seed, h, w):
    g = np.random.default_rng(seed)
    return g.integers(0, 256, size=(h, w, 3), dtype=np.uint8)


def test_to_tensor_and_geometry():
    u8 = u8_image(1, 37, 53)
    x = A.to_tensor(u8, "cuda")
    ref = R.to_tensor(torch.from_numpy(u8))
    assert torch.equal(x.cpu(), ref)
    for k in (1, -1, 2):
        assert torch.equal(A.rot90(x, k).cpu(), torch.rot90(ref, k, [1, 2]))
    assert torch.equal(A.hflip(x).cpu(), torch.flip(ref, [2]))
    assert torch.equal(A.vflip(x).cpu(), torch.flip(ref, [1]))


@pytest.mark.parametrize("op,factors", [
    ("brightness", (0.6, 1.0, 1.37)), ("contrast", (0.9, 1.08)), ("saturation", (0.6, 1.4)),
    ("hue", (-0.1, -0.03, 0.0, 0.07, 0.1)),
])
def test_color_ops(op, factors):
    x = A.to_tensor(u8_image(2, 41, 29), "cuda")
    xc = x.cpu()
    fn = {"brightness": (A.adjust_brightness, R.adjust_brightness), "contrast": (A.adjust_contrast, R.adjust_contrast),
          "saturation": (A.adjust_saturation, R.adjust_saturation), "hue": (A.adjust_hue, R.adjust_hue)}[op]
    for f in factors:
        assert rel_inf(fn[0](x, f), fn[1](xc, f)) <= 2e-5, (op, f)
    # non-quantised input too (values strictly inside (0, 1) and a few > 1 before clamping)
    y = torch.rand(3, 16, 24) * 1.1
    for f in factors:
        assert rel_inf(fn[0](y.cuda(), f), fn[1](y, f)) <= 2e-5, (op, f)


def test_grayscale():
    x = torch.rand(3, 20, 30)
    assert rel_inf(A.rgb_to_grayscale3(x.cuda()), R.rgb_to_grayscale(x, 3)) <= 1e-6


@pytest.mark.parametrize("hw,size", [((96, 160), (64, 64)), ((53, 77), (128, 160)), ((512, 384), (96, 160)),
                                     ((31, 47), (31, 47)), ((200, 90), (160, 96))])
def test_resize(hw, size):
    x = torch.rand(3, *hw)
    assert rel_inf(A.resize(x.cuda(), size), R.resize(x, size)) <= 2e-5


def test_resized_crop():
    x = torch.rand(3, 120, 90)
    for (t, l, h, w) in ((10, 5, 60, 70), (0, 0, 120, 90), (33, 41, 17, 29)):
        assert rel_inf(A.resized_crop(x.cuda(), t, l, h, w, (96, 128)), R.resized_crop(x, t, l, h, w, (96, 128))) <= 2e-5


@pytest.mark.parametrize("k", [3, 5, 7, 9])
def test_gaussian_blur(k):
    x = torch.rand(3, 33, 47)
    for sigma in (0.1, 0.77, 2.0):
        assert rel_inf(A.gaussian_blur(x.cuda(), k, sigma), R.gaussian_blur(x, k, sigma)) <= 2e-5


def _oracle_ops():
    """A CPU stand-in for augment.py built from the oracle, so data_loader's own classes (and
    their random draws) run once on each side."""
    return types.SimpleNamespace(
        to_tensor=lambda img, dev: R.to_tensor(torch.from_numpy(np.asarray(img))),
        rot90=lambda x, k: torch.rot90(x, k, [1, 2]), hflip=lambda x: torch.flip(x, [2]),
        vflip=lambda x: torch.flip(x, [1]), adjust_brightness=R.adjust_brightness,
        adjust_contrast=R.adjust_contrast, adjust_saturation=R.adjust_saturation, adjust_hue=R.adjust_hue,
        rgb_to_grayscale3=lambda x: R.rgb_to_grayscale(x, 3).contiguous(), resize=R.resize,
        resized_crop=R.resized_crop, gaussian_blur=R.gaussian_blur)


def test_get_transform_pipeline_seeded(monkeypatch):
    """data_loader.get_transform end to end (every branch exercised over 40 draws) vs the same
    classes running the oracle ops under the same seeds."""
    imgs = [u8_image(100 + i, 90 + 7 * (i % 10), 120 - 5 * (i % 10)) for i in range(40)]
    outs = []
    for ops in (A, _oracle_ops()):
        monkeypatch.setattr(DL, "A", ops)
        random.seed(5)
        torch.manual_seed(5)
        tr = DL.get_transform(True, (96, 128))
        for t in tr.transforms:   # raise the probabilities so every transform fires regularly
            if hasattr(t, "p"):
                t.p = 0.6 if not isinstance(t, DL.RandomResizeOrCrop) else 0.5
        outs.append([tr(im) for im in imgs])
    for i, (a, b) in enumerate(zip(*outs)):
        assert a.shape == b.shape == (3, 96, 128)
        assert rel_inf(a, b) <= 1e-4, i
