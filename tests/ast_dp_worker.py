"""Worker of tests/test_gpu_ast_train.py::test_ast_trainer_dp_uneven_matches_single_process
(launched by torch.distributed.run, 2 ranks, gloo -- both ranks share the box's one GPU): one
data-parallel ASTTrainer step (train.py:186-300 under sharding) with an uneven 2 + 1 shard of a
global batch of 3. SyncBatchNorm over the train-mode encoder, shard-weighted loss terms, the SUM
all-reduce of the gradient arena (AdaAttN / BN gradients are copied into it). Rank 0 saves the
reduced gradients, the updated parameters and the BN running statistics. argv: out_path"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbitrarystyletransfer_amd import dp, models, synth  # noqa: E402
from arbitrarystyletransfer_amd.train import ASTTrainer, default_ast_args  # noqa: E402

GLOBAL_BATCH, SIZE = 3, 64


def inputs():
    c = torch.from_numpy(synth.image(961, (GLOBAL_BATCH, 3, SIZE, SIZE)))
    s = torch.from_numpy(synth.image(962, (GLOBAL_BATCH, 3, SIZE, SIZE)))
    return c, s


ATT_SCALE = 0.125   # as test_ast_trainer_step_golden: W_q, W_k scaled after the live init (diffuse attention)


def make_trainer(device, hook):
    torch.manual_seed(0)
    ast = models.AST(attention=True).load_live_init()
    with torch.no_grad():
        for att in (ast.ada_att_1, ast.ada_att_2):
            att.W_q.weight.mul_(ATT_SCALE)
            att.W_k.weight.mul_(ATT_SCALE)
    return ASTTrainer(default_ast_args(batch_size=GLOBAL_BATCH), device=device, ast=ast, grad_hook=hook)


def main(out_path):
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    content, style = inputs()
    a, b = dp.shard_range(GLOBAL_BATCH, rank, world)
    snap = {}
    tr = make_trainer("cuda:0", lambda ps: snap.update({n: p.grad.detach().clone() for n, p in tr.ast.named_parameters()}))
    assert tr.grad_arena is not None and tr.world == world
    out = tr.train_step(content[a:b].cuda(), style[a:b].cuda(), record=True)
    if rank == 0:
        res = {"grad_norm": float(out["grad_norm"]), "content_loss_logged": tr.train_dict["content_loss"][-1]}
        for n, p in tr.ast.named_parameters():
            res[f"grad:{n}"] = snap[n].cpu().numpy()
            res[f"param:{n}"] = p.detach().cpu().numpy()
        for n, buf in tr.ast.named_buffers():
            res[f"buf:{n}"] = buf.detach().cpu().numpy()
        np.savez(out_path, **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
