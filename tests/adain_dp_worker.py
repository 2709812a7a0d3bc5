"""Worker of tests/test_gpu_training.py::test_adain_dp_two_ranks_match_single_process (launched by
torch.distributed.run): one data-parallel AdaIN training step (BASELINE.json config 4 semantics,
train.py:287-300 under sharding) of AdaINTrainer + dp.FlatGradArena on the HIP kernels. Each rank
takes its shard of the global batch; rank 0 saves the reduced gradients (snapshot between the
all-reduce and clip + Adam) and the updated parameters. Both ranks share the box's one GPU, so the
collective runs on gloo (staged through the host); with one rank per GPU bench.py uses RCCL.
argv: out_path global_batch size [full]"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbitrarystyletransfer_amd import dp, synth  # noqa: E402
from arbitrarystyletransfer_amd.train import AdaINTrainer, default_args  # noqa: E402


def main(out_path, global_batch, size, full):
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    content = torch.from_numpy(synth.image(941, (global_batch, 3, size, size)))
    style = torch.from_numpy(synth.image(942, (global_batch, 3, size, size)))
    a, b = dp.shard_range(global_batch, rank, world)
    snap = {}

    def hook(params):
        snap["grads"] = [p.grad.detach().clone() for p in params]

    tr = AdaINTrainer(default_args(batch_size=global_batch, full_losses=full), device="cuda:0", grad_hook=hook)
    assert tr.grad_arena is not None and tr.world == world
    out = tr.train_step(content[a:b].cuda(), style[a:b].cuda())
    for p in tr.params:   # the reduced gradient is the arena (no copy for kernel-written slices)
        assert p.grad.data_ptr() == tr.grad_arena.view_for(p).data_ptr()
    if rank == 0:
        res = {"grad_norm": float(out["grad_norm"])}
        for i, (g, p) in enumerate(zip(snap["grads"], tr.params)):
            res[f"grad{i}"] = g.cpu().numpy()
            res[f"param{i}"] = p.detach().cpu().numpy()
        np.savez(out_path, **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), len(sys.argv) > 4 and sys.argv[4] == "full")
