#!/usr/bin/env python3
"""Phase timing of the split-bf16 conv (conv3x3_x3_kernel<M16>) from in-kernel clock stamps.

Diagnostic only: needs the X3_STAMP build (bash scripts/build_variants.sh stamp "-DX3_STAMP=1"
conv3x3_igemm.hip), which this script selects through AST_HIP_LIB. The stamps never reach an output.
python scripts/x3_stamps.py OUTDIR [cfg n cin h w cout up pad pool]
Writes OUTDIR/x3_stamps_<shape>.npz (raw records) and prints the per-phase summary
(scripts/x3_stamps_summary.py does the same from the npz)."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("AST_HIP_LIB", os.path.join(ROOT, "build_var", "libast_hip_stamp.so"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from arbitrarystyletransfer_amd import _lib, ops, synth  # noqa: E402
import x3_stamps_summary as S  # noqa: E402

out = sys.argv[1]
args = sys.argv[2:] if len(sys.argv) > 2 else ["28", "16", "256", "128", "128", "256", "1", "zeros", "0"]
cfg = int(args[0])
n, cin, h, w, cout, up = (int(v) for v in args[1:7])
pad, pool = args[7], args[8] == "1"
dev = torch.device("cuda")
lib = _lib.lib()
fn = lib.ast_dbg_x3_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
x = torch.from_numpy(synth.image(5, (n, cin, h, w))).to(dev)
wp = ops.pack_conv3x3(torch.from_numpy(synth.conv_weight(6, cout, cin, 3)).to(dev))
b = torch.from_numpy(synth.conv_bias(7, cout)).to(dev)


def run():
    ops.conv3x3(x, wp, b, cout, upsample=up, pad_mode=pad, want_pre=not pool, want_act=False, want_pool=pool, cfg=cfg)


t0 = time.time()
while time.time() - t0 < 2.0:  # back-to-back launches so the clock settles (MI355X_MICROARCH.md DVFS item 6)
    for _ in range(10):
        run()
    torch.cuda.synchronize()
_lib.check(fn(None, 0, 1), "stamp clear")
run()
torch.cuda.synchronize()
NWG, REC = 2048, 200
buf = np.zeros(NWG * 16 * REC, dtype=np.uint32)
_lib.check(fn(buf.ctypes.data, buf.nbytes, 0), "stamp read")
tag = f"c{cfg}_{n}x{cin}x{h}x{w}_{cout}_up{up}_{pad}{'_pool' if pool else ''}"
os.makedirs(out, exist_ok=True)
np.savez_compressed(os.path.join(out, f"x3_stamps_{tag}.npz"), rec=buf.reshape(NWG, 16, REC))
print(tag)
S.summary(buf.reshape(NWG, 16, REC))
