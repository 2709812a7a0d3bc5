"""torch.ops.ast_hip.*: the hot ops registered as PyTorch custom operators ("What
the C++ side exports"), for callers that want the dispatcher (torch.compile / fake-tensor tracing,
TorchScript, `torch.ops` lookups) rather than the ctypes binding. Same kernels, same C ABI: the
registration shim csrc/torch_ops.cpp (libast_torch_ops.so) calls the entry points of
include/ast_hip.h on PyTorch's current HIP stream; Meta kernels give output shapes.

    from arbitrarystyletransfer_amd import torch_ops
    ops = torch_ops.load()
    out = ops.adain(content, style, 1.0, True)                 # models.py:43-51 (+ blend, :471)
    mean, std = ops.channel_stats(x, True, 0.0)                # model_util.py:3-8
    pre, act, pool = ops.conv3x3_fwd(x, ops.conv3x3_pack(w), b, cout, 1, 0, None, None,
                                     False, True, False, -1)  # unrequested outputs are empty
    g = ops.gram(feat)                                         # losses.py:105-109
"""
from __future__ import annotations

import os

import torch

from . import _lib

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libast_torch_ops.so")
OPS = ("adain", "channel_stats", "conv3x3_pack", "conv3x3_fwd", "gram")
_loaded = False


def load():
    """Register the ops (once) and return the torch.ops.ast_hip namespace; raises if the shim was
    not built (no fallback)."""
    global _loaded
    if not _loaded:
        if not os.path.exists(LIB_PATH):
            raise _lib.HipOpError(f"{LIB_PATH} is missing: build it first "
                                  "(python -c 'import __graft_entry__ as g; g.build()')")
        _lib.lib()   # the C-ABI library first (the shim resolves its symbols from the same copy)
        torch.ops.load_library(LIB_PATH)
        _loaded = True
    return torch.ops.ast_hip
