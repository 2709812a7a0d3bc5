"""Worker of tests/test_gpu_mbtrain.py::test_autoencoder_dp_syncbn_step_golden (launched by
torch.distributed.run, 2 ranks): one data-parallel AutoEncoder training step with SyncBatchNorm,
each rank on its shard of the golden batch; rank 0 saves what the test compares. Both ranks share
the box's one GPU, so the collectives run on gloo (staged through the host)."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbitrarystyletransfer_amd import dp, models  # noqa: E402
from arbitrarystyletransfer_amd.train import AutoencoderTrainer, default_ae_args  # noqa: E402


def main(out_path):
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ae_train_step_64.npz"))
    content = torch.from_numpy(g["content"])
    a, b = dp.shard_range(content.shape[0], rank, world)
    poison = os.environ.get("AST_POISON")
    if poison:   # debugging aid: fill the caching allocator's free blocks so unwritten reads show
        big = [torch.full((1 << 28,), float(poison), device="cuda:0") for _ in range(4)]
        mid = [torch.full((1 << 22,), float(poison), device="cuda:0") for _ in range(64)]
        small = [torch.full((1 << 16,), float(poison), device="cuda:0") for _ in range(1024)]
        del big, mid, small
    tr = AutoencoderTrainer(default_ae_args(batch_size=content.shape[0]), device="cuda:0", model=models.AutoEncoder().load_live_init())
    assert tr.grad_arena is not None
    snap = {}
    orig = tr.ae_optim.step

    def step():
        snap.update({n: p.grad.detach().clone() for n, p in tr.model.named_parameters()})
        orig()

    tr.ae_optim.step = step
    out = tr.train_step(content[a:b].cuda())
    losses = torch.stack([out[k].detach().float() for k in ("recon_loss", "content_loss", "loss")]).cpu()
    dist.all_reduce(losses)
    losses /= world
    recon = [torch.zeros_like(out["recon"]).cpu() for _ in range(world)]
    dist.all_gather(recon, out["recon"].detach().cpu().contiguous())
    if rank == 0:
        props = torch.cuda.get_device_properties(0)
        res = {"losses": losses.numpy(), "recon": torch.cat(recon).numpy(), "grad_norm": float(out["grad_norm"]),
               "cus": props.multi_processor_count, "gcn": str(getattr(props, "gcnArchName", ""))}
        for n, p in tr.model.named_parameters():
            res[f"grad:{n}"] = snap[n].cpu().numpy()
            res[f"param:{n}"] = p.detach().cpu().numpy()
        for n, buf in tr.model.named_buffers():
            res[f"buf:{n}"] = buf.detach().cpu().numpy()
        np.savez(out_path, **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
