"""Worker of tests/test_gpu_rccl.py (a fresh child process, started before it touches the GPU):
executes the RCCL ("nccl") branches of dp.py on the box's one GPU in a world of 1 and compares
each against the same computation without a process group:
  * AdaINTrainer step (config 4 semantics, train.py:287-300): FlatGradArena SUM all-reduce;
  * FlatGradArena AVG all-reduce (DDP semantics);
  * AutoencoderTrainer step with SyncBatchNorm: all_gather_into_tensor of the per-channel
    (count, mean, M2) and the all-reduce of the backward sums;
  * broadcast_style_stats (one-style-many-contents).
A world of 1 makes every collective an identity, so results must agree bitwise with the
no-process-group run (the merge of one part is the single-process merge). argv: out_json"""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arbitrarystyletransfer_amd import dp, models, synth  # noqa: E402
from arbitrarystyletransfer_amd.train import (AdaINTrainer, AutoencoderTrainer, default_ae_args,  # noqa: E402
                                              default_args)


def adain_step(dev, c, s):
    torch.manual_seed(0)
    snap = {}
    tr = AdaINTrainer(default_args(batch_size=c.shape[0]), device=dev,
                      grad_hook=lambda ps: snap.update(g=[p.grad.detach().clone() for p in ps]))
    out = tr.train_step(c, s, record=True)
    return tr, snap["g"] + [p.detach().clone() for p in tr.params] + [out["grad_norm"].reshape(1)]


def ae_step(dev, c):
    torch.manual_seed(0)
    tr = AutoencoderTrainer(default_ae_args(batch_size=c.shape[0]), device=dev,
                            model=models.AutoEncoder().load_live_init())
    snap = {}
    orig = tr.ae_optim.step

    def step():
        snap["g"] = [p.grad.detach().clone() for p in tr.model.parameters()]
        orig()
    tr.ae_optim.step = step
    out = tr.train_step(c, record=True)
    return tr, (snap["g"] + [p.detach().clone() for p in tr.model.parameters()] +
                [b.detach().clone() for b in tr.model.buffers()] + [out["recon"].detach(), out["grad_norm"].reshape(1)])


def compare(name, a, b, report):
    assert len(a) == len(b), name
    worst, bitwise = 0.0, True
    for x, y in zip(a, b):
        x, y = x.float(), y.float()
        bitwise = bitwise and torch.equal(x, y)
        worst = max(worst, float((x - y).abs().max() / y.abs().max().clamp_min(1e-30)))
    report[name] = {"bitwise": bitwise, "rel_inf": worst}
    assert worst <= 1e-6, (name, worst)


def main(out_json):
    dev = torch.device("cuda:0")
    c = torch.from_numpy(synth.image(951, (2, 3, 64, 64))).to(dev)
    s = torch.from_numpy(synth.image(952, (2, 3, 64, 64))).to(dev)
    report = {}
    # without a process group (the single-process path)
    tr0, ref_adain = adain_step(dev, c, s)
    assert tr0.grad_arena is None
    _, ref_ae = ae_step(dev, c)
    net = models.AdaINStyleTransfer().to(dev).eval()
    with torch.no_grad():
        sm, ss = net.style_statistics(s)
    # the same under RCCL, world of 1
    dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    tr1, got_adain = adain_step(dev, c, s)
    assert tr1.grad_arena is not None and not tr1.grad_arena.average   # SUM (shard-weighted losses)
    for p in tr1.params:
        assert p.grad.data_ptr() == tr1.grad_arena.view_for(p).data_ptr()
    compare("adain_trainer_sum", got_adain, ref_adain, report)
    report["train_dict"] = {k: v for k, v in tr1.train_dict.items() if v}
    assert tr1.train_dict["content_loss"] == tr0.train_dict["content_loss"]
    # AVG mode: an arena over the same parameters, all-reduced in place
    arena = dp.FlatGradArena(tr1.params, average=True)
    arena.unregister()
    arena.flat.copy_(torch.linspace(-3, 5, arena.flat.numel(), device=dev))
    before = arena.flat.clone()
    for p in tr1.params:
        p.grad = arena.view_for(p)
    arena.all_reduce()
    compare("arena_avg", [arena.flat], [before], report)
    # SyncBatchNorm AutoEncoder step: all_gather_into_tensor + all_reduce_sum of the BN sums
    tr2, got_ae = ae_step(dev, c)
    assert tr2.grad_arena is not None
    assert all(dp.sync_group(m) is not None for m in tr2.model.modules() if isinstance(m, torch.nn.BatchNorm2d))
    compare("ae_syncbn_step", got_ae, ref_ae, report)
    # style statistics broadcast from rank 0
    with torch.no_grad():
        bm, bs = dp.broadcast_style_stats(sm.clone(), ss.clone(), src=0)
    compare("broadcast_style_stats", [bm, bs], [sm, ss], report)
    torch.cuda.synchronize()
    dist.destroy_process_group()
    with open(out_json, "w") as f:
        json.dump(report, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
