"""conv3x3 configs 24-31 vs torch's conv2d on shapes of the decoder dgrad / forward (AST_CONV_M16=2:
every config runs as requested)."""
import os
import sys

os.environ["AST_CONV_M16"] = "2"
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from arbitrarystyletransfer_amd import ops  # noqa: E402

torch.manual_seed(0)
dev = "cuda"
shapes = [(2, 256, 18, 20, 256, 1), (2, 512, 10, 12, 256, 1), (2, 256, 8, 8, 256, 2), (2, 128, 34, 36, 128, 1),
          (2, 256, 16, 16, 128, 1), (2, 64, 66, 68, 64, 1), (3, 128, 18, 20, 64, 1), (2, 256, 18, 20, 128, 1)]
for (n, cin, h, w, cout, up) in shapes:
    x = torch.randn(n, cin, h, w, device=dev)
    wt = torch.randn(cout, cin, 3, 3, device=dev) * 0.05
    b = torch.randn(cout, device=dev)
    xu = F.interpolate(x, scale_factor=up, mode="nearest") if up > 1 else x
    ref = F.conv2d(xu.double(), wt.double(), b.double(), padding=1).float()
    packed = ops.pack_conv3x3(wt)
    line = []
    for cfg in range(24, 32):
        try:
            pre, _, _ = ops.conv3x3(x, packed, b, cout, upsample=up, want_pre=True, want_act=False, cfg=cfg, _pack=False)
            err = ((pre - ref).abs().max() / ref.abs().max()).item()
            line.append(f"{cfg}:{err:.1e}")
        except Exception as e:  # noqa: BLE001
            line.append(f"{cfg}:-({str(e)[:20]})")
    print((n, cin, h, w, cout, up), " ".join(line), flush=True)
