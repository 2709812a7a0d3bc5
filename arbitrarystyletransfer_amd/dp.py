"""Data parallelism for the training step (BASELINE.json config 4): one process per GPU,
batch-sharded, gradients reduced by a single all-reduce over xGMI (torch.distributed "nccl" =
RCCL on ROCm).

Whenever a default process group is initialised the trainers take this path, at any world size:
a world of 1 runs the same collectives (trivial on one rank), which is how the RCCL branches are
exercised on a one-GPU box (tests/test_gpu_rccl.py).

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
    """[start, stop) of this rank's images; shards differ by at most one image. Every rank must
    get at least one image (an empty shard would reach the kernels with n = 0)."""
    if global_batch < world:
        raise ValueError(f"global batch {global_batch} < world size {world}: some rank would get no image")
    base, extra = divmod(global_batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard_weight(global_batch: int, rank: int, world: int) -> float:
    """local / global image count: the factor a rank's batch-mean loss terms carry so that the
    SUM over ranks of the per-rank gradients is the full-batch gradient for uneven shards too."""
    a, b = shard_range(global_batch, rank, world)
    return (b - a) / global_batch


def active() -> bool:
    """True when a default process group is initialised (the data-parallel path is taken)."""
    return dist.is_available() and dist.is_initialized()


def is_main() -> bool:
    """Rank 0, or no process group: the process that writes checkpoints and logs."""
    return not active() or dist.get_rank() == 0


def barrier() -> None:
    if active():
        dist.barrier()


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
    backward kernels write into it, and reduces it across ranks in one all-reduce: a SUM for the
    trainers (each rank's loss terms already carry their shard weight, so the sum is the
    full-batch gradient, uneven shards included), or an AVG (average=True, DDP semantics)."""

    def __init__(self, params, device=None, average=True):
        self.params = list(params)
        device = device or self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(total, device=device, dtype=torch.float32)
        self.slices = {}
        off = 0
        for p in self.params:
            self.slices[id(p)] = (off, p.numel(), tuple(p.shape))
            off += p.numel()
        # average=True: AVG over ranks (equal shards, per-rank batch-mean losses: DDP). False: SUM,
        # for trainers whose per-rank losses are already weighted by shard_weight (exact for
        # uneven shards)
        self.average = average
        self._taken = set()
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

    def take(self, p):
        """The arena slice for a weight-gradient kernel to write p's gradient into, or None when
        it must not: the slice was already handed out in this backward (p used twice in the
        graph) or p already holds an accumulated gradient. Reset by all_reduce / reset."""
        if id(p) in self._taken or p.grad is not None:
            return None
        self._taken.add(id(p))
        return self.view_for(p)

    def reset(self):
        self._taken.clear()

    def all_reduce(self, group=None):
        """Reduce the arena across the group in place (AVG, or SUM when average=False).
        Parameters whose .grad is not a view of the arena (produced by a non-HIP op, or the sum
        of two contributions) are copied in first."""
        self._taken.clear()
        for p in self.params:
            if p.grad is not None and p.grad.data_ptr() != self.view_for(p).data_ptr():
                self.view_for(p).copy_(p.grad)
                p.grad = self.view_for(p)
        if not active():
            return
        if dist.get_backend(group) == "nccl":
            dist.all_reduce(self.flat, op=dist.ReduceOp.AVG if self.average else dist.ReduceOp.SUM, group=group)
        else:  # gloo (CPU tests; device tensors staged through the host) has no AVG
            all_reduce_sum(self.flat, group)
            if self.average:
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


# ------------------------------------------------------------------------------------------------
# SyncBatchNorm for data-parallel AutoEncoder training: the reference
# trains with batch statistics over its whole batch (train_autoencoder.py, BatchNorm2d in train
# mode), so a batch-sharded step must merge the statistics over ranks. Forward: every rank's
# per-channel (count, mean, M2) in double, [c][3], is all-gathered (W*c*24 bytes) and merged on
# device (Chan's update); backward: the per-channel sums (dy, dy*xhat) are all-reduced for the
# input gradient, while dgamma/dbeta stay local: each rank's are the gradient of its own
# shard-weighted loss, and the gradient all-reduce SUMS them into the full-batch gradient.
# ------------------------------------------------------------------------------------------------
def convert_sync_batchnorm(module: torch.nn.Module, group=None) -> torch.nn.Module:
    """Mark every BatchNorm2d of `module` for cross-rank statistics (mbtrain.BatchNormTrainFn);
    the counterpart of torch.nn.SyncBatchNorm.convert_sync_batchnorm."""
    for m in module.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m._ast_sync = True
            m._ast_sync_group = group
    return module


def sync_group(bn):
    """The process group a BatchNorm syncs over, or None (not marked / not distributed)."""
    if not getattr(bn, "_ast_sync", False) or not active():
        return None
    return getattr(bn, "_ast_sync_group", None) or dist.group.WORLD


def _staged(t, group):
    """gloo moves host tensors only: stage a device tensor through the host for it."""
    return t.cpu() if dist.get_backend(group) == "gloo" and t.device.type != "cpu" else t


def all_gather_bn_stats(stats: torch.Tensor, group=None) -> torch.Tensor:
    """[c][3] double per rank -> [W][c][3] on stats' device."""
    world = dist.get_world_size(group)
    src = _staged(stats.contiguous(), group)
    out = torch.empty((world,) + tuple(stats.shape), dtype=stats.dtype, device=src.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, src, group=group)
    else:
        dist.all_gather(list(out.unbind(0)), src, group=group)
    return out.to(stats.device)


def global_terms(terms: dict, weights: dict, group=None) -> dict:
    """Full-batch values of per-rank loss terms, for logging: sum over ranks of weight * term (the
    shard weight for batch-mean terms, 1 for batch-sum terms such as tv). One all-reduce of a
    small stacked vector; in a single process the terms come back unchanged."""
    keys = sorted(terms)
    if not active():
        return {k: terms[k] for k in keys}
    vec = torch.stack([terms[k].detach().float().reshape(()) * weights.get(k, 1.0) for k in keys])
    all_reduce_sum(vec, group)
    return {k: vec[i] for i, k in enumerate(keys)}


def all_reduce_sum(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place sum over ranks (staged through the host for gloo)."""
    src = _staged(t, group)
    dist.all_reduce(src, op=dist.ReduceOp.SUM, group=group)
    if src is not t:
        t.copy_(src)
    return t
