"""Per-kernel timing of representative config-5 blocks (bf16, B=32): expand_dw and pw launch time,
depthwise FMA rate and dw-output write rate. python scripts/bench_mb_blocks.py [batch]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbitrarystyletransfer_amd import ops, synth  # noqa: E402
from arbitrarystyletransfer_amd.mobilenetv2 import DepthWiseConv  # noqa: E402

# name, inp, oup, stride, expand, k, use_norm, h, up
CASES = [
    ("enc1 16->16 t6 k3 1024", 16, 16, 1, 6, 3, True, 1024, 1),
    ("enc2 16->24 t6 k3 s2 1024", 16, 24, 2, 6, 3, True, 1024, 1),
    ("enc4 24->40 t6 k5 s2 512", 24, 40, 2, 6, 5, True, 512, 1),
    ("dec8 40->40 t4 k5 1024", 40, 40, 1, 4, 5, False, 1024, 1),
    ("dec10 40->24 t6 k5 1024", 40, 24, 1, 6, 5, False, 1024, 1),
    ("dec11 24->24 t6 k3 1024", 24, 24, 1, 6, 3, False, 1024, 1),
    ("dec7up 40->40 r1 k3 512->1024", 40, 40, 1, 1, 3, False, 512, 2),
    ("enc8 80->80 t4 k3 128", 80, 80, 1, 4, 3, True, 128, 1),
    ("enc11 96->96 t3 k5 128", 96, 96, 1, 3, 5, True, 128, 1),
]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    only = sys.argv[2] if len(sys.argv) > 2 else None
    dev = torch.device("cuda:0")
    res = {}
    for name, inp, oup, s, t, k, norm, h, up in CASES:
        if only and not name.startswith(only):
            continue
        blk = synth.live_init_(DepthWiseConv(inp, oup, s, t, kernel_size=k, use_norm=norm), 3).eval().to(dev)
        blk = blk.to(torch.bfloat16)
        x = torch.rand(B, inp, h, h, device=dev).to(torch.bfloat16)
        with torch.no_grad():
            for _ in range(2):
                blk.run(x, None, up)
            torch.cuda.synchronize()
            timer = ops.LaunchTimer()
            with timer:
                for _ in range(5):
                    y = blk.run(x, None, up)
            torch.cuda.synchronize()
        ed = [ms for tag, _, ms in timer.results() if tag.startswith("mb expand_dw")]
        pw = [ms for tag, _, ms in timer.results() if tag.startswith("mb pw")]
        ho = y.shape[2]
        hid = blk.hidden_dim
        fma = B * hid * ho * ho * k * k
        dbytes = B * hid * ho * ho * 2
        e, p = sum(ed) / len(ed), sum(pw) / len(pw)
        res[name] = {"expand_dw_ms": round(e, 3), "pw_ms": round(p, 3),
                     "dw_tfma_s": round(fma / e / 1e9, 2), "d_write_gbs": round(dbytes / e / 1e6, 1),
                     "pw_d_read_gbs": round(dbytes / p / 1e6, 1)}
        print(name, res[name], flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/mb_blocks.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
