"""Drop-in for the reference data_loader.py with the augmentation on the GPU (SURVEY.md §8f
"next" #3). Same names and call structure (Random90Rot, ConditionalResize, RandomResizeOrCrop,
RandomBlur, ImageTransform, get_transform, image_loader, infinite_sampler,
InfiniteSamplerWrapper, FlatFolderDataset, FlatFolderDatasetAE); images are decoded on the host
(PIL), their uint8 bytes are copied to the device once, and every transform after ToTensor runs
as a HIP kernel (augment.py / csrc/augment.hip) on the [C, H, W] fp32 device tensor.

The random draws follow the reference's transforms (Python `random` for the reference's own
classes, torch's RNG where torchvision draws: RandomHorizontalFlip / RandomVerticalFlip /
RandomApply / RandomGrayscale use torch.rand(1), ColorJitter torch.randperm(4) + uniform_,
RandomResizedCrop.get_params, GaussianBlur's sigma), so a seeded run draws the same parameters
in the same order. Decoding stays on the host: the image has no JPEG decoder on the device.
"""
from __future__ import annotations

import math
import random
from pathlib import Path

import torch
import torch.utils.data as data

from . import augment as A
from .conf import device, img_sizes  # noqa: F401

try:  # PIL decodes on the host, as in the reference (data_loader.py:5, :186)
    from PIL import Image
except ImportError:  # pragma: no cover - PIL is in the image
    Image = None


class Compose:
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, x):
        for t in self.transforms:
            x = t(x)
        return x


class ToTensor:
    """transforms.ToTensor, on the device (uint8 upload + conversion kernel)."""

    def __init__(self, dev=None):
        self.device = dev

    def __call__(self, img):
        dev = self.device or (device if device != "cpu" else "cuda")
        return A.to_tensor(img.convert("RGB") if hasattr(img, "convert") else img, dev)


class Random90Rot:
    """data_loader.py:14-24."""

    def __init__(self, p=0.5):
        self.p = p

    def __call__(self, x):
        if random.random() <= self.p:
            rot_dir = random.choice([-1, 1])
            x = A.rot90(x, rot_dir)
        return x


class RandomHorizontalFlip:
    def __init__(self, p=0.5):
        self.p = p

    def __call__(self, x):
        return A.hflip(x) if torch.rand(1) < self.p else x


class RandomVerticalFlip:
    def __init__(self, p=0.5):
        self.p = p

    def __call__(self, x):
        return A.vflip(x) if torch.rand(1) < self.p else x


class ColorJitter:
    """transforms.ColorJitter(brightness, contrast, saturation, hue): adjustments in a random
    order (torch.randperm(4)) with uniformly drawn factors."""

    def __init__(self, brightness=0, contrast=0, saturation=0, hue=0):
        self.brightness = (max(0.0, 1 - brightness), 1 + brightness) if brightness else None
        self.contrast = (max(0.0, 1 - contrast), 1 + contrast) if contrast else None
        self.saturation = (max(0.0, 1 - saturation), 1 + saturation) if saturation else None
        self.hue = (-hue, hue) if hue else None

    def get_params(self):
        fn_idx = torch.randperm(4)
        b = None if self.brightness is None else float(torch.empty(1).uniform_(*self.brightness))
        c = None if self.contrast is None else float(torch.empty(1).uniform_(*self.contrast))
        s = None if self.saturation is None else float(torch.empty(1).uniform_(*self.saturation))
        h = None if self.hue is None else float(torch.empty(1).uniform_(*self.hue))
        return fn_idx, b, c, s, h

    def __call__(self, img):
        fn_idx, b, c, s, h = self.get_params()
        for fn_id in fn_idx.tolist():
            if fn_id == 0 and b is not None:
                img = A.adjust_brightness(img, b)
            elif fn_id == 1 and c is not None:
                img = A.adjust_contrast(img, c)
            elif fn_id == 2 and s is not None:
                img = A.adjust_saturation(img, s)
            elif fn_id == 3 and h is not None:
                img = A.adjust_hue(img, h)
        return img


class RandomApply:
    def __init__(self, transforms, p=0.5):
        self.transforms = transforms
        self.p = p

    def __call__(self, img):
        if self.p < torch.rand(1):
            return img
        for t in self.transforms:
            img = t(img)
        return img


class Resize:
    """transforms.Resize((h, w)) on a tensor (antialiased bilinear)."""

    def __init__(self, size):
        self.size = size

    def __call__(self, x):
        return A.resize(x, self.size)


class RandomResizedCrop:
    """transforms.RandomResizedCrop(size, scale=(0.08, 1), ratio=(3/4, 4/3))."""

    def __init__(self, size, scale=(0.08, 1.0), ratio=(3.0 / 4.0, 4.0 / 3.0)):
        self.size = size
        self.scale = scale
        self.ratio = ratio

    @staticmethod
    def get_params(img, scale, ratio):
        height, width = int(img.shape[-2]), int(img.shape[-1])
        area = height * width
        log_ratio = torch.log(torch.tensor(ratio))
        for _ in range(10):
            target_area = area * torch.empty(1).uniform_(scale[0], scale[1]).item()
            aspect_ratio = torch.exp(torch.empty(1).uniform_(log_ratio[0], log_ratio[1])).item()
            w = int(round(math.sqrt(target_area * aspect_ratio)))
            h = int(round(math.sqrt(target_area / aspect_ratio)))
            if 0 < w <= width and 0 < h <= height:
                i = torch.randint(0, height - h + 1, size=(1,)).item()
                j = torch.randint(0, width - w + 1, size=(1,)).item()
                return i, j, h, w
        in_ratio = float(width) / float(height)
        if in_ratio < min(ratio):
            w = width
            h = int(round(w / min(ratio)))
        elif in_ratio > max(ratio):
            h = height
            w = int(round(h * max(ratio)))
        else:
            w, h = width, height
        return (height - h) // 2, (width - w) // 2, h, w

    def __call__(self, img):
        i, j, h, w = self.get_params(img, self.scale, self.ratio)
        return A.resized_crop(img, i, j, h, w, self.size)


class GaussianBlur:
    """transforms.GaussianBlur(kernel_size, sigma=(0.1, 2.0))."""

    def __init__(self, kernel_size, sigma=(0.1, 2.0)):
        self.kernel_size = kernel_size
        self.sigma = sigma

    def __call__(self, img):
        sigma = torch.empty(1).uniform_(self.sigma[0], self.sigma[1]).item()
        return A.gaussian_blur(img, self.kernel_size, sigma)


class RandomGrayscale:
    def __init__(self, p=0.1):
        self.p = p

    def __call__(self, img):
        return A.rgb_to_grayscale3(img) if torch.rand(1) < self.p else img


class ConditionalResize:
    """data_loader.py:27-45: resize to at least min_size on the short side."""

    def __init__(self, min_size=256):
        self._min_size = min_size

    def __call__(self, tensor):
        if tensor.shape[1] < self._min_size or tensor.shape[2] < self._min_size:
            if tensor.shape[1] < tensor.shape[2]:
                new_width = self._min_size
                new_height = int(tensor.shape[2] / tensor.shape[1] * new_width)
            else:
                new_height = self._min_size
                new_width = int(tensor.shape[1] / tensor.shape[2] * new_height)
            tensor = A.resize(tensor, [new_width, new_height])   # Resize([a, b]) = (h=a, w=b), as :41
        return tensor


class RandomResizeOrCrop:
    """data_loader.py:47-70."""

    def __init__(self, imsize, p=0.90):
        self.p = p
        self.resize = Resize((imsize[0], imsize[1]))
        self.cond_resize = ConditionalResize(min(imsize[0], imsize[1]))
        self.rand_crop_resize = RandomResizedCrop((imsize[0], imsize[1]))

    def __call__(self, x):
        if random.random() < self.p:
            x = self.resize(x)
        else:
            x = self.cond_resize(x)
            x = self.rand_crop_resize(x)
        return x


class RandomBlur:
    """data_loader.py:72-84."""

    def __init__(self, p=0.1, blur_sizes=[3, 5, 7, 9]):
        self.p = p
        self.blur_sizes = blur_sizes

    def __call__(self, x):
        if random.random() <= self.p:
            blur_fac = random.choice(self.blur_sizes)
            self.blur = GaussianBlur(blur_fac)
            x = self.blur(x)
        return x


class ImageTransform:
    """data_loader.py:87-107: a new random output size every 2*batch_size images."""

    def __init__(self, batch_size, use_transform=True):
        self.batch_size = batch_size
        self.transform = get_transform(use_transform)
        self.num_in_batch = 0

    def reset(self):
        self.num_in_batch = 0
        rand_h = random.choice(img_sizes)
        rand_w = random.choice(img_sizes)
        self.transform = get_transform(True, (rand_h, rand_w))

    def __call__(self, img):
        if self.num_in_batch >= self.batch_size * 2:
            self.reset()
        self.num_in_batch += 1
        return self.transform(img)


def get_transform(crop=True, imsize=(256, 256)):
    """data_loader.py:110-135, every step after ToTensor on the device."""
    if crop:
        return Compose([
            ToTensor(),
            Random90Rot(0.25),
            RandomHorizontalFlip(0.25),
            RandomVerticalFlip(0.25),
            RandomApply([ColorJitter(0.4, 0.10, 0.4, 0.10)], p=0.25),
            RandomResizeOrCrop(imsize),
            RandomBlur(0.05),
            RandomGrayscale(p=0.001),
        ])
    return Compose([ToTensor(), Resize((imsize, 256))])


def image_loader(image_name):
    """data_loader.py:137-141."""
    image = Image.open(image_name)
    image = get_transform(False)(image).unsqueeze(0)
    return image.to(torch.float)


def infinite_sampler(n):
    i = 0
    perm = torch.randperm(n).tolist()
    while True:
        yield perm[i]
        i += 1
        if i >= n:
            i = 0
            perm = torch.randperm(n).tolist()


class InfiniteSamplerWrapper(data.sampler.Sampler):
    def __init__(self, data_source):
        self.num_samples = len(data_source)

    def __iter__(self):
        return iter(infinite_sampler(self.num_samples))

    def __len__(self):
        return 2 ** 31


class FlatFolderDataset(data.Dataset):
    """data_loader.py:162-200 (items are device tensors: iterate in the main process, num_workers=0)."""

    def __init__(self, content_root, style_root, transform=None):
        super().__init__()
        self.content_paths = self._get_paths(content_root)
        self.style_paths = self._get_paths(style_root)
        self.transform = transform

    def _get_paths(self, root):
        paths = []
        for d in root:
            paths += list(Path(d).glob('*'))
        random.shuffle(paths)
        return paths

    def _get_item(self, paths):
        idx = torch.randint(0, len(paths), ())
        while True:
            try:
                img = Image.open(str(paths[idx])).convert("RGB")
                if self.transform is not None:
                    img = self.transform(img).float()
                return img
            except Exception as e:  # the reference retries another image (data_loader.py:190-192)
                print("e:", e)
                idx = torch.randint(0, len(paths), ())

    def _decode(self, paths):
        """The host half of _get_item: a random image of `paths` decoded to a uint8 RGB HWC array
        (what a DataLoader worker returns; the device half is the transform, in the trainer process)."""
        import numpy as np
        idx = torch.randint(0, len(paths), ())
        while True:
            try:
                return np.asarray(Image.open(str(paths[idx])).convert("RGB"))
            except Exception as e:  # as _get_item: retry another image
                print("e:", e)
                idx = torch.randint(0, len(paths), ())

    def __getitem__(self, idx):
        return self._get_item(self.content_paths), self._get_item(self.style_paths)

    def __len__(self):
        return len(self.content_paths) + len(self.style_paths)

    def name(self):
        return 'FlatFolderDataset'


class FlatFolderDatasetAE(FlatFolderDataset):
    """data_loader.py:202-236."""

    def __init__(self, content_root, transform=None):
        data.Dataset.__init__(self)
        self.content_paths = self._get_paths(content_root)
        self.transform = transform

    def __getitem__(self, idx):
        return self._get_item(self.content_paths)

    def __len__(self):
        return len(self.content_paths)


# ------------------------------------------------------------------------------------------------
# Parallel host decoding (the reference's DataLoader(num_workers=4 | 8), train.py:66-75,
# train_autoencoder.py:188-195): worker processes open and decode images (PIL, CPU only); the
# trainer process uploads them and runs ToTensor and every augmentation as HIP kernels, so the GPU is
# used by one process only. Workers are forked when the iterator is built before the process touches
# the GPU (the helpers below start their workers at once), as the reference builds its loaders first;
# spawned otherwise.
# ------------------------------------------------------------------------------------------------

class HostDecoded(data.Dataset):
    """DataLoader-worker view of a FlatFolderDataset / FlatFolderDatasetAE: item = decoded uint8
    arrays, a (content, style) pair or a content image, drawn at random as the dataset's own
    __getitem__ does (data_loader.py:184-197, :221-233)."""

    def __init__(self, dataset):
        self.ds = dataset

    def __getitem__(self, idx):
        if isinstance(self.ds, FlatFolderDatasetAE):
            return self.ds._decode(self.ds.content_paths)
        return self.ds._decode(self.ds.content_paths), self.ds._decode(self.ds.style_paths)

    def __len__(self):
        return len(self.ds)


def _collate_list(batch):
    return batch


def device_batches(decoded_iter, transform, pairs=True):
    """Batches of the device transform over decoded items: (content, style) stacked [B, 3, H, W]
    pairs, or content batches. ImageTransform keeps one output size for 2 * batch_size images,
    so a batch stacks (data_loader.py:87-107)."""
    for items in decoded_iter:
        if pairs:
            yield (torch.stack([transform(c).float() for c, _ in items]),
                   torch.stack([transform(st).float() for _, st in items]))
        else:
            yield torch.stack([transform(c).float() for c in items])


def _gpu_initialized():
    return torch.cuda.is_initialized()


def _decoded_loader(dataset, batch_size, num_workers):
    # forked workers (the default start) only while this process has not initialised the GPU: a fork
    # of a HIP-initialised process is not safe, so a caller that touched the GPU first gets spawned
    # workers (they import the package and decode with PIL only)
    ctx = "spawn" if num_workers > 0 and _gpu_initialized() else None
    loader = data.DataLoader(HostDecoded(dataset), batch_size=batch_size, sampler=InfiniteSamplerWrapper(dataset),
                             num_workers=num_workers, collate_fn=_collate_list, multiprocessing_context=ctx,
                             persistent_workers=num_workers > 0, prefetch_factor=2 if num_workers > 0 else None)
    # iter() starts the workers now: forked when the caller builds the iterator before touching the GPU
    # (as the trainers do), spawned (a fresh interpreter importing this package, no GPU init) otherwise
    return iter(loader)


def content_style_iter(content_dir, style_dir, transform, batch_size, num_workers=4):
    """train.py:66-75: an endless iterator of (content, style) device batches, decoded by
    `num_workers` host processes and transformed on the device (transform: e.g. ImageTransform)."""
    ds = FlatFolderDataset(content_dir, style_dir, transform=None)
    return device_batches(_decoded_loader(ds, batch_size, num_workers), transform, pairs=True)


def content_iter(content_dir, transform, batch_size, num_workers=8):
    """train_autoencoder.py:188-195: the AutoEncoder trainer's content batches, likewise."""
    ds = FlatFolderDatasetAE(content_dir, transform=None)
    return device_batches(_decoded_loader(ds, batch_size, num_workers), transform, pairs=False)
