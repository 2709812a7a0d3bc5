"""Time ops.adaattn (fp32 / bf16) at AST shapes; prints TFLOP/s of the whole op (6*C*Nq*Nk per
image: S = K Q^T plus P [V, V^2]) against the fp32 / bf16 MFMA peaks."""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from arbitrarystyletransfer_amd import ops  # noqa: E402

PEAK = {torch.float32: 157.3, torch.bfloat16: 2516.6}


def run(n, c, h, w, dtype=torch.float32, iters=5):
    x = torch.rand(n, c, h, w, device="cuda", dtype=dtype)
    y = torch.rand(n, c, h, w, device="cuda", dtype=dtype)
    wts = [torch.randn(c, c, device="cuda") * (0.15 / c ** 0.5) for _ in range(3)]
    ops.adaattn(x, y, *wts)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        ops.adaattn(x, y, *wts)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / iters
    fl = 6.0 * n * c * (h * w) ** 2
    tf = fl / ms / 1e9
    print(f"adaattn {str(dtype)[6:]} n={n} c={c} {h}x{w}: {ms:.3f} ms  {tf:.1f} TFLOP/s  "
          f"{100 * tf / PEAK[dtype]:.1f}% of peak", flush=True)


if __name__ == "__main__":
    if "--big-bf16" in sys.argv:   # one config-5-sized call (PMC runs)
        run(32, 128, 128, 128, torch.bfloat16, iters=1)
        sys.exit(0)
    if "--big-f32" in sys.argv:
        run(32, 128, 128, 128, torch.float32, iters=1)
        sys.exit(0)
    dts = [torch.float32] + ([torch.bfloat16] if "--bf16" in sys.argv else [])
    for dt in dts:
        run(1, 128, 64, 64, dt)
        run(8, 128, 64, 64, dt)
        run(4, 128, 128, 128, dt)
        run(32, 128, 128, 128, dt, iters=2)
        run(32, 128, 128, 128, dt, iters=2)
