"""Time the MobileNet training 1x1-conv GEMM (mbtrain.gemm -> ast_mbt_gemm_f32) on the dominant
AE/AST trainer shapes and report effective HBM GB/s: forward (M = cout, K = cin, N = images x
pixels, image folded into N) over K, M and N, to separate per-tile overhead from streaming rate."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from arbitrarystyletransfer_amd import mbtrain  # noqa: E402

dev = torch.device("cuda:0")


def run(M, K, imgs, P, reps=20):
    x = torch.randn(imgs, K, P, device=dev)
    w = torch.randn(M, K, device=dev)
    y = torch.empty(imgs, M, P, device=dev)
    args = (w, x, y, M, imgs * P, K, 1, (0, K, 1), (K * P, P, 1), (M * P, P, 1))
    for _ in range(3):
        mbtrain.gemm(*args, fold_n=P)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        mbtrain.gemm(*args, fold_n=P)
    e.record()
    e.synchronize()
    ms = s.elapsed_time(e) / reps
    gb = 4 * (K * imgs * P + M * imgs * P) / 1e9
    print(f"M={M:4d} K={K:4d} imgs={imgs:3d} P={P:6d}: {ms * 1e3:8.1f} us  {gb / ms * 1e3:7.0f} GB/s  "
          f"{2 * M * K * imgs * P / ms / 1e9:7.1f} TF", flush=True)


for M, K in [(16, 96), (24, 144), (144, 24), (96, 16), (16, 16), (64, 64), (128, 128)]:
    run(M, K, 16, 25600)
for imgs in (4, 64):
    run(16, 96, imgs, 25600)
for P in (1600, 6400, 102400):
    run(16, 96, 16, P)
