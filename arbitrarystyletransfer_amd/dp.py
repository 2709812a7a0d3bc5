"""Data parallelism for the training step (BASELINE.json config 4): one process per GPU,
batch-sharded, gradients averaged by a single all-reduce over xGMI (torch.distributed "nccl" =
RCCL on ROCm).

The trainable parameters' gradients live in one flat fp32 arena: the HIP weight-gradient kernel
writes each dW/db straight into its slice (functional.GRAD_ARENA), autograd adopts those views as
.grad without a copy, and the whole 14 MB decoder gradient is reduced in one collective (a ring
all-reduce is per-link bound: 2*(W-1)/W * 14 MB / ~150 GB/s ~ 0.2 ms, against a ~100 ms step;
bucketing/overlap would not pay here). Forward-only stylisation needs no collective at all.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from . import functional


def shard_range(global_batch: int, rank: int, world: int):
    """[start, stop) of this rank's images; shards differ by at most one image."""
    base, extra = divmod(global_batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def init_from_env(backend=None, device=None):
    """Initialise the default process group from torchrun's env (RANK/WORLD_SIZE/MASTER_*)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1 and not dist.is_initialized():
        backend = backend or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl" and device is not None:
            dist.init_process_group(backend, device_id=device)
        else:
            dist.init_process_group(backend)
    return rank, world


class FlatGradArena:
    """One contiguous gradient buffer for `params`; registers each parameter's slice so the
    backward kernels write into it, and averages it across ranks in one all-reduce."""

    def __init__(self, params, device=None):
        self.params = list(params)
        device = device or self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(total, device=device, dtype=torch.float32)
        self.slices = {}
        off = 0
        for p in self.params:
            self.slices[id(p)] = (off, p.numel(), tuple(p.shape))
            off += p.numel()
        self.register()

    def register(self):
        for p in self.params:
            functional.GRAD_ARENA[id(p)] = self

    def unregister(self):
        for p in self.params:
            functional.GRAD_ARENA.pop(id(p), None)

    def view_for(self, p):
        off, n, shape = self.slices[id(p)]
        return self.flat[off:off + n].view(shape)

    def all_reduce(self, group=None):
        """Average the arena across the group (in place). Parameters whose .grad is not a view
        of the arena (e.g. produced by a non-HIP op) are copied in first."""
        for p in self.params:
            if p.grad is not None and p.grad.data_ptr() != self.view_for(p).data_ptr():
                self.view_for(p).copy_(p.grad)
                p.grad = self.view_for(p)
        if not dist.is_initialized() or dist.get_world_size(group) == 1:
            return
        if dist.get_backend(group) == "nccl":
            dist.all_reduce(self.flat, op=dist.ReduceOp.AVG, group=group)
        else:  # gloo (CPU tests) has no AVG
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)
            self.flat.div_(dist.get_world_size(group))

    def __call__(self, params=None):
        self.all_reduce()


def broadcast_style_stats(style_mean, style_std, src: int = 0, group=None):
    """One-style-many-contents mode: the rank owning the style image computed
    its relu4_1 statistics (AdaINStyleTransfer.style_statistics); every rank receives them in one
    broadcast of a packed [2, ...] tensor (2*512 fp32 = 4 KB). Other ranks pass tensors of the
    same shape (contents ignored). Returns (mean, std) on every rank."""
    packed = torch.stack([style_mean.reshape(-1), style_std.reshape(-1)]).contiguous()
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(packed, src=src, group=group)
    return packed[0].view_as(style_mean), packed[1].view_as(style_std)
