"""Throughput of the get_transform pipeline (data_loader.py:110-135): the device path
(arbitrarystyletransfer_amd.data_loader, uint8 upload + HIP kernels) vs the same classes on the CPU
oracle ops (torchvision's tensor formulas with torch CPU ops), on pre-decoded 512x512 RGB images
(PIL decoding is host work in both). Prints one JSON line."""
import json
import os
import random
import sys
import time
import types

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbitrarystyletransfer_amd import augment as A  # noqa: E402
from arbitrarystyletransfer_amd import data_loader as DL  # noqa: E402
from oracle import ref_augment as R  # noqa: E402


def run(ops, imgs, n, sync):
    DL.A = ops
    random.seed(0)
    torch.manual_seed(0)
    tr = DL.get_transform(True, (256, 256))
    for im in imgs[:4]:
        tr(im)
    sync()
    t0 = time.perf_counter()
    for i in range(n):
        tr(imgs[i % len(imgs)])
    sync()
    return n / (time.perf_counter() - t0)


def main():
    g = np.random.default_rng(0)
    imgs = [g.integers(0, 256, size=(512, 512, 3), dtype=np.uint8) for _ in range(16)]
    gpu = run(A, imgs, 400, torch.cuda.synchronize)
    cpu_ops = types.SimpleNamespace(
        to_tensor=lambda img, dev: R.to_tensor(torch.from_numpy(np.asarray(img))),
        rot90=lambda x, k: torch.rot90(x, k, [1, 2]), hflip=lambda x: torch.flip(x, [2]),
        vflip=lambda x: torch.flip(x, [1]), adjust_brightness=R.adjust_brightness,
        adjust_contrast=R.adjust_contrast, adjust_saturation=R.adjust_saturation, adjust_hue=R.adjust_hue,
        rgb_to_grayscale3=lambda x: R.rgb_to_grayscale(x, 3).contiguous(), resize=R.resize,
        resized_crop=R.resized_crop, gaussian_blur=R.gaussian_blur)
    threads = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    torch.set_num_threads(threads)
    cpu = run(cpu_ops, imgs, 100, lambda: None)
    print(json.dumps({"workload": "get_transform(crop=True, (256, 256)) on 512x512 uint8 RGB images (decoded)",
                      "device_images_per_s": gpu, "cpu_images_per_s": cpu, "cpu_threads": threads,
                      "note": "per-image launches (batch 1); PIL decode excluded on both sides"}))


if __name__ == "__main__":
    main()
