#!/usr/bin/env python3
"""Benchmark: stylised images/s for the VGG19-relu4_1 AdaIN forward (BASELINE.json config 2:
bs=8 per GPU, 512x512, fp32) on MI355X, one process per GPU.

A step = one forward pass over one batch: encode 8 content + 8 style images (one launch per
conv layer, both batches together), AdaIN + blend, decode 8 images. Inputs and weights are
synthetic (live-init recipe, arbitrarystyletransfer_amd/synth.py) and resident in HBM before the
timed region. N > 1 GPUs: each rank stylises its own batch of 8 (the path shards by image, no
collective on the data path) -> weak scaling; value = all ranks' images / max-over-ranks time.

Prints ONE JSON line (rank 0). Extra objects:
  roofline      dominant kernel (conv3x3 MFMA-fp32 implicit GEMM, all 18 launches of a step):
                algorithmic FLOPs / summed kernel time from HIP events recorded on the launch
                stream during the timed steps, against the 157.3 TF fp32 matrix peak.
  cpu_baseline  the CPU oracle (oracle/ref_cpu.py, stock torch CPU ops = the reference's CPU
                path) on a bounded sample (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from arbitrarystyletransfer_amd import models, ops, synth  # noqa: E402

METRIC = "stylised images/sec at 512x512 bs=8, 1->8 MI355X; encoder MFMA %-of-peak"
PEAK_FP32_MFMA_TF = 157.3       # MI355X_MICROARCH.md: 256 CU x 4 SIMD x 64 FLOP/clk x 2.4 GHz
PEAK_HBM_GBS = 8000.0
PEAK_BF16_MFMA_TF = 2516.6      # dense bf16 MFMA (MI355X_MICROARCH.md), no sparsity
# The VGG convs run on the split-bf16 MFMA kernel: every fp32 product is 6 bf16 MFMA products
# (x = hi + mid + lo exactly), so the ceiling of its fp32-accurate work is the bf16
# peak / 6 = 419.4 TFLOP/s, 2.67x the 157.3 TF fp32 matrix peak.
PEAK_SPLIT_BF16_TF = PEAK_BF16_MFMA_TF / 6


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=None, help="images per GPU (config 2: 8, config 5: 32)")
    p.add_argument("--size", type=int, default=None, help="image side (config 2: 512, config 5: 1024)")
    p.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU-baseline time budget (0 = skip)")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="0 = best of os.cpu_count(), the affinity/cgroup CPU share and OMP_NUM_THREADS")
    p.add_argument("--mode", choices=["fwd", "train", "mobilenet", "ae-train", "ast-train"], default="fwd",
                   help="fwd: config 2 (the headline metric); train: config 3/4 AdaIN training step; "
                        "mobilenet: config 5; ae-train: train_autoencoder.py step (SURVEY §8f next #4); "
                        "ast-train: train.py's ASTTrainer step (MobileNet AST + AdaAttN)")
    p.add_argument("--full-losses", action="store_true",
                   help="train mode: add train.py's hist, org_img and out_of_range terms (SURVEY §8f next #2)")
    p.add_argument("--attention", action="store_true",
                   help="mobilenet mode: stylise with the reference AST's AdaAttN (SURVEY §8f next #1) "
                        "instead of AdaIN")
    return p.parse_args()


def train_bench(args, dev, rank, world):
    """Config 3 (bs=16, 1 GPU) / config 4 (bs=8 per GPU, RCCL gradient all-reduce): one step =
    forward, loss network x3, losses, backward, all-reduce (N>1), clip + Adam."""
    from arbitrarystyletransfer_amd.train import AdaINTrainer, default_args
    B, S = args.batch or 16, args.size or 512
    # args.batch_size = the global batch; the trainer shards it (dp.shard_range), keeps the decoder
    # gradient in one flat arena and sums it across ranks in one all-reduce before clip + Adam
    trainer = AdaINTrainer(default_args(batch_size=B * world, image_size=S, full_losses=args.full_losses),
                           device=dev)
    assert (trainer.grad_arena is not None) == (world > 1)
    content = torch.from_numpy(synth.image(777 + 2 * rank, (B, 3, S, S))).to(dev)
    style = torch.from_numpy(synth.image(778 + 2 * rank, (B, 3, S, S))).to(dev)
    for _ in range(args.warmup):
        trainer.train_step(content, style)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    timer = ops.LaunchTimer()
    t0 = time.perf_counter()
    with timer:
        for _ in range(args.steps):
            out = trainer.train_step(content, style)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], device=dev if dist.get_backend() == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert torch.isfinite(out["loss"]), "non-finite loss"
    recs = timer.results()
    mm = [(tag, fl, ms) for tag, fl, ms in recs if tag.startswith(("conv3x3", "wgrad"))]
    fl = sum(f for _, f, _ in mm)
    ms = sum(m for _, _, m in mm)
    tf = fl / (ms * 1e-3) / 1e12
    wg = [(f, m) for tag, f, m in mm if tag.startswith("wgrad")]
    wg_tf = sum(f for f, _ in wg) / (sum(m for _, m in wg) * 1e-3) / 1e12 if wg else None
    # every matrix-core kernel of the step: the convs and wgrads above plus the loss Gram matrices
    # and their backward (v_mfma_f32_32x32x2f32, csrc/losses.hip)
    ms_gram = sum(m for tag, _, m in recs if tag.startswith(("gram ", "gram_bwd ")))
    result = {
        "metric": "AdaIN training images/sec at 512x512 (config 3: bs=16/GPU; config 4: batch-sharded)",
        "value": B * world * args.steps / elapsed, "unit": "images/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (live-init weights, U[0,1) images), resident in HBM",
        "config": {"workload": f"AdaIN train step (decoder trained; VGG loss network to relu_15; content+style+"
                               f"lf+tv{'+hist+org_img+out_of_range' if args.full_losses else ''} losses; "
                               f"clip 2.0 + Adam), bs={B}/GPU {S}x{S} fp32",
                   "global_batch": B * world, "image_size": S, "parallelism": f"data-parallel x{world}"},
        "roofline": {"bound": "mfma", "kernel": "conv3x3 fwd/dgrad + wgrad MFMA launches of a step (split-bf16)",
                     "achieved": tf, "peak": PEAK_SPLIT_BF16_TF, "unit": "TFLOP/s", "frac": tf / PEAK_SPLIT_BF16_TF,
                     "peak_basis": "fp32-accurate ceiling of the split-bf16 kernels: dense bf16 MFMA / 6",
                     "fp32_mfma_peak": PEAK_FP32_MFMA_TF, "frac_of_fp32_mfma_peak": tf / PEAK_FP32_MFMA_TF,
                     "traffic": None, "wgrad_tflops": wg_tf,
                     "mfma_share_of_step": ms / args.steps / (elapsed / args.steps * 1e3),
                     "matrix_kernels_share_of_step": (ms + ms_gram) / args.steps / (elapsed / args.steps * 1e3),
                     "mfma_tflop_per_step": fl / args.steps / 1e12},
    }
    if rank == 0 and world == 1 and args.cpu_seconds > 0 and not args.full_losses:
        result["cpu_baseline"] = cpu_baseline_train(S, args.cpu_seconds, cpu_thread_options(args.cpu_threads))
    if rank == 0:
        print(json.dumps(result), flush=True)


def ae_train_bench(args, dev, rank, world):
    """AutoEncoder training step (train_autoencoder.py:124-165): the MobileNet
    AutoEncoder in training mode (BatchNorm batch statistics), reconstruction + perceptual Huber
    losses through the frozen VGG loss network, backward, clip 10 + Adam. bs=16 at 160x160 (the
    reference's batch size and its largest training size, conf.py img_sizes). N > 1: data parallel,
    bs=16 per rank (weak scaling), SyncBatchNorm (all-gather of per-rank BN statistics, all-reduce
    of the backward sums) and one gradient all-reduce over RCCL before clip + Adam."""
    from arbitrarystyletransfer_amd.train import AutoencoderTrainer, default_ae_args
    B, S = args.batch or 16, args.size or 160
    trainer = AutoencoderTrainer(default_ae_args(batch_size=B * world), device=dev,
                                 model=models.AutoEncoder().load_live_init())
    content = torch.from_numpy(synth.image(901 + rank, (B, 3, S, S))).to(dev)
    for _ in range(args.warmup):
        trainer.train_step(content, record=False)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = trainer.train_step(content, record=False)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], device=dev if dist.get_backend() == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert torch.isfinite(out["loss"]), "non-finite loss"
    # per-kernel-family times: HIP events around every launch of further steps, outside the timed
    # region (the eager step is host-issue-bound, so two events per launch would inflate it)
    ksteps = 3
    timer = ops.LaunchTimer()
    with timer:
        for _ in range(ksteps):
            trainer.train_step(content, record=False)
    torch.cuda.synchronize(dev)
    fam = {}
    for tag, fl, ms in timer.results():
        k = tag.split()[0]
        f0, m0, c0 = fam.get(k, (0.0, 0.0, 0))
        fam[k] = (f0 + fl, m0 + ms, c0 + 1)
    mm = [fam[k] for k in fam if k.startswith(("conv3x3", "wgrad"))]
    fl, ms = sum(f for f, _, _ in mm), sum(m for _, m, _ in mm)
    tf = fl / (ms * 1e-3) / 1e12 if ms else 0.0
    result = {
        "metric": "AutoEncoder training images/sec (train_autoencoder.py step)",
        "value": B * world * args.steps / elapsed, "unit": "images/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (live-init weights, U[0,1) images), resident in HBM",
        "config": {"workload": f"AutoEncoder train step (MobileNet encoder/decoder, BatchNorm train mode; recon + "
                               f"perceptual Huber via VGG relu_1..relu_15; clip 10 + Adam), bs={B}/GPU {S}x{S} fp32",
                   "global_batch": B * world, "image_size": S,
                   "parallelism": f"data-parallel x{world}" + (" + SyncBatchNorm" if world > 1 else "")},
        "roofline": {"bound": "mfma", "kernel": "loss-network conv3x3 fwd/dgrad launches of a step (split-bf16)",
                     "achieved": tf, "peak": PEAK_SPLIT_BF16_TF, "unit": "TFLOP/s", "frac": tf / PEAK_SPLIT_BF16_TF,
                     "fp32_mfma_peak": PEAK_FP32_MFMA_TF, "frac_of_fp32_mfma_peak": tf / PEAK_FP32_MFMA_TF,
                     "traffic": None, "mfma_share_of_step": ms / ksteps / (elapsed / args.steps * 1e3),
                     "timing_source": "HIP events around each launch of 3 eager steps after the timed ones"},
        "kernels_ms_per_step": {k: round(m / ksteps, 4) for k, (f, m, c) in sorted(fam.items())},
        "mbgemm_tflops": (fam["mbgemm"][0] / (fam["mbgemm"][1] * 1e-3) / 1e12) if "mbgemm" in fam else None,
    }
    if rank == 0:
        print(json.dumps(result), flush=True)


def ast_train_bench(args, dev, rank, world):
    """The reference's own trainer step, ASTTrainer (train.py:186-300; SURVEY §8f next #1 with
    its caller): the MobileNet AST with AdaAttN in training mode, the four VGG loss-network
    passes, every train.py loss term, backward through decoder / ada_out / AdaAttN / encoder,
    clip 2.0 + Adam over ast.parameters(). bs=8 (train.py:408) at 160x160 (the largest of
    conf.py img_sizes). N > 1: data parallel, bs=8 per rank, SyncBatchNorm + one gradient
    all-reduce."""
    from arbitrarystyletransfer_amd.train import ASTTrainer, default_ast_args
    B, S = args.batch or 8, args.size or 160
    # hipGraph replay in one process; eager under data parallelism (ASTTrainer's default there)
    graph = os.environ.get("AST_TRAIN_GRAPH", "1" if world == 1 else "0") != "0"
    trainer = ASTTrainer(default_ast_args(batch_size=B * world), device=dev,
                         ast=models.AST(attention=True).load_live_init(), graph=graph)
    content = torch.from_numpy(synth.image(905 + rank, (B, 3, S, S))).to(dev)
    style = torch.from_numpy(synth.image(925 + rank, (B, 3, S, S))).to(dev)
    for _ in range(args.warmup):   # the first step captures the hipGraph (graph mode)
        trainer.train_step(content, style, record=False)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = trainer.train_step(content, style, record=False)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], device=dev if dist.get_backend() == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert torch.isfinite(out["loss"]), "non-finite loss"
    # per-kernel-family times: HIP events around every launch of an eager step (a replayed graph
    # launches nothing from Python), same kernels and shapes as the timed steps
    eager = ASTTrainer(default_ast_args(batch_size=B * world), device=dev,
                       ast=models.AST(attention=True).load_live_init(), graph=False)
    ksteps = 3
    eager.train_step(content, style, record=False)
    torch.cuda.synchronize(dev)
    timer = ops.LaunchTimer()
    te = time.perf_counter()
    with timer:
        for _ in range(ksteps):
            eager.train_step(content, style, record=False)
    torch.cuda.synchronize(dev)
    eager_ms = (time.perf_counter() - te) / ksteps * 1e3
    del eager
    fam = {}
    for tag, fl, ms in timer.results():
        k = tag.split()[0]
        f0, m0, c0 = fam.get(k, (0.0, 0.0, 0))
        fam[k] = (f0 + fl, m0 + ms, c0 + 1)
    mm = [fam[k] for k in fam if k.startswith(("conv3x3", "wgrad"))]
    fl, ms = sum(f for f, _, _ in mm), sum(m for _, m, _ in mm)
    tf = fl / (ms * 1e-3) / 1e12 if ms else 0.0
    args.steps, steps_timed = ksteps, args.steps   # the per-step kernel figures below are per eager step
    result = {
        "metric": "AST training images/sec (train.py ASTTrainer step, MobileNet AST + AdaAttN)",
        "value": B * world * steps_timed / elapsed, "unit": "images/s", "n_gpus": world, "steps": steps_timed,
        "warmup": args.warmup, "ms_per_step": elapsed / steps_timed * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (live-init weights, U[0,1) images), resident in HBM",
        "step_mode": "hipGraph replay (train.StepGraph)" if graph else "eager",
        "eager_ms_per_step": eager_ms,
        "config": {"workload": f"ASTTrainer step (MobileNet AST + AdaAttN in train mode; content, style, lf, tv, hist, "
                               f"org_img, out_of_range losses via the VGG loss network; clip 2.0 + Adam), "
                               f"bs={B}/GPU {S}x{S} fp32",
                   "global_batch": B * world, "image_size": S,
                   "parallelism": f"data-parallel x{world}" + (" + SyncBatchNorm" if world > 1 else "")},
        "roofline": {"bound": "mfma", "kernel": "loss-network conv3x3 fwd/dgrad launches of a step (split-bf16)",
                     "achieved": tf, "peak": PEAK_SPLIT_BF16_TF, "unit": "TFLOP/s", "frac": tf / PEAK_SPLIT_BF16_TF,
                     "fp32_mfma_peak": PEAK_FP32_MFMA_TF, "frac_of_fp32_mfma_peak": tf / PEAK_FP32_MFMA_TF,
                     "traffic": None, "mfma_share_of_step": ms / args.steps / (elapsed / steps_timed * 1e3),
                     "timing_source": "HIP events around each launch of 3 eager steps of the same shapes"},
        "kernels_ms_per_step": {k: round(m / args.steps, 4) for k, (f, m, c) in sorted(fam.items())},
        "mbgemm_tflops": (fam["mbgemm"][0] / (fam["mbgemm"][1] * 1e-3) / 1e12) if "mbgemm" in fam else None,
    }
    if rank == 0:
        print(json.dumps(result), flush=True)


def _pmc_traffic(name):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 FETCH_SIZE /
    WRITE_SIZE passes (profiles/<name>, scripts/pmc_traffic.py), and where that number comes from.
    PMC counters cannot be collected inside this timed run; the value is replayed from the named
    profile, taken on the commit it records: (None, None) when absent."""
    try:
        with open(os.path.join(ROOT, "profiles", name)) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    return d.get("hbm_bytes_per_launch"), f"profiles/{name}@{d.get('commit', 'unknown')} ({d.get('source', '')})"


def mobilenet_bench(args, dev, rank, world):
    """Config 5: MobileNet-style variant (Encoder x2 -> AdaIN@[12,14] -> ada_out -> Decoder,
    exporting), bs=32/GPU at 1024x1024, bf16 storage with fp32 arithmetic. The roofline is HBM:
    SURVEY.md §8d's block-fused minimum traffic (each block reads its input and writes its output
    once) per step / step time, against 8 TB/s; `kernels` breaks the step down per kernel family."""
    from arbitrarystyletransfer_amd import mobilenetv2
    B, S = args.batch or 32, args.size or 1024
    bf = torch.bfloat16
    net = models.AST(exporting=True, attention=args.attention).load_live_init().eval().to(dev).to(bf)
    content = torch.from_numpy(synth.image(821 + 2 * rank, (B, 3, S, S))).to(dev).to(bf)
    style = torch.from_numpy(synth.image(822 + 2 * rank, (B, 3, S, S))).to(dev).to(bf)

    def step():
        with torch.no_grad():
            return net(content, style)

    mobilenetv2.IO_TRACE, mobilenetv2.DW_TRACE = [], []
    out = step()
    fused_min_bytes = sum(mobilenetv2.IO_TRACE)
    dw_fma_per_step = sum(mobilenetv2.DW_TRACE)
    mobilenetv2.IO_TRACE = mobilenetv2.DW_TRACE = None
    for _ in range(max(0, args.warmup - 1)):
        out = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    timer = ops.LaunchTimer()
    t0 = time.perf_counter()
    with timer:
        for _ in range(args.steps):
            out = step()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], device=dev if dist.get_backend() == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert torch.isfinite(out.float()).all(), "non-finite output"
    recs = timer.results()
    fam = {}
    attn = [0.0, 0.0, 0]
    for tag, nb, ms in recs:
        if tag.startswith("adaattn"):   # FLOP-tagged (MFMA-bound), not byte-tagged
            attn[0] += nb
            attn[1] += ms
            attn[2] += 1
            continue
        key = tag.split(" ")[0] + " " + tag.split(" ")[1]
        a = fam.setdefault(key, [0.0, 0.0, 0])
        a[0] += -nb
        a[1] += ms
        a[2] += 1
    kernels = {k: {"ms_per_step": v[1] / args.steps, "launches_per_step": v[2] // args.steps,
                   "algorithmic_gbs": v[0] / (v[1] * 1e-3) / 1e9} for k, v in fam.items()}
    if attn[2]:
        tf = attn[0] / (attn[1] * 1e-3) / 1e12
        kernels["adaattn bf16"] = {"ms_per_step": attn[1] / args.steps, "launches_per_step": attn[2] // args.steps,
                                   "tflops": tf, "frac_of_bf16_mfma_peak": tf / PEAK_BF16_MFMA_TF}
    step_s = elapsed / args.steps
    achieved = fused_min_bytes / step_s / 1e9
    # PMC bytes per expand_dw launch, measured at the default B=32, 1024^2
    mb_traffic = _pmc_traffic("mb_traffic.json") if (B, S) == (32, 1024) and not args.attention else (None, None)
    step_pmc = (None, None)
    if (B, S) == (32, 1024) and not args.attention:
        try:
            with open(os.path.join(ROOT, "profiles", "r06k_mb_step_traffic.json")) as f:
                d = json.load(f)
            step_pmc = (d["hbm_gb_per_step"], "profiles/r06k_mb_step_traffic.json (" + d["source"] + ")")
        except (OSError, ValueError, KeyError):
            pass
    ed = fam.get("mb expand_dw")
    ed_gbs = (ed[0] / (ed[1] * 1e-3) / 1e9) if ed else None
    dw_tf = (2 * dw_fma_per_step * args.steps / (ed[1] * 1e-3) / 1e12) if ed else None
    result = {
        "metric": "stylised images/sec, MobileNet variant bs=32 1024x1024 bf16 (config 5)"
                  + (", AdaAttN stylisation" if args.attention else ""),
        "value": B * world * args.steps / elapsed, "unit": "images/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": step_s * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (live-init MobileNet weights, U[0,1) images), resident in HBM",
        "config": {"workload": f"config 5: MobileNet-style Encoder (content+style) -> "
                               f"{'AdaAttN' if args.attention else 'AdaIN'}@[12,14] -> ada_out -> "
                               f"Decoder(exporting), bs={B}/GPU {S}x{S}, bf16 storage / fp32 accumulate",
                   "global_batch": B * world, "image_size": S, "parallelism": f"batch-sharded x{world}"},
        # dominant kernel: the fused expand + depthwise launches (~60% of the step); algorithmic bytes
        # = its input read + depthwise-output write. The depthwise runs on the VALU (v4) or, for the k5
        # blocks with cin <= 48, as a Toeplitz product on the bf16 MFMA (v5, csrc/mb_ed5.hip); "valu"
        # gives the depthwise MAC rate of the family against the 157.3 TF fp32 vector peak.
        "roofline": {"bound": "hbm", "kernel": "mb expand_dw (expand 1x1 MFMA + depthwise kxk on VALU (v4) or "
                                               "Toeplitz MFMA (v5 k5), all launches)",
                     "achieved": ed_gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": (ed_gbs / PEAK_HBM_GBS) if ed_gbs else None,
                     # PMC bytes per expand_dw launch, measured at the default B=32, 1024^2
                     "traffic": mb_traffic[0], "traffic_source": mb_traffic[1],
                     "avg_launch_ms": (ed[1] / ed[2]) if ed else None,
                     "avg_launch_gb": (ed[0] / ed[2] / 1e9) if ed else None,
                     "valu": {"dw_tflops": dw_tf, "peak": PEAK_FP32_MFMA_TF,
                              "frac": (dw_tf / PEAK_FP32_MFMA_TF) if dw_tf else None},
                     "whole_step": {"fused_min_gb_per_step": fused_min_bytes / 1e9, "achieved_gbs": achieved,
                                    "frac": achieved / PEAK_HBM_GBS,
                                    # every dispatch's FETCH_SIZE x2 + WRITE_SIZE per step, committed PMC run
                                    "pmc_gb_per_step": step_pmc[0], "pmc_source": step_pmc[1]},
                     "kernel_share_of_step": sum(m for _, _, m in recs) / args.steps / (step_s * 1e3)},
        "kernels": kernels,
    }
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        result["cpu_baseline"] = cpu_baseline_mobilenet(S, args.cpu_seconds, cpu_thread_options(args.cpu_threads),
                                                        args.attention)
    if rank == 0:
        print(json.dumps(result), flush=True)


def _cpu_model():
    import platform
    cpu_model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return f"{cpu_model}, {platform.machine()}"


def _usable_cpus():
    """CPUs this process may run on: the affinity mask and the cgroup v2 quota (None if unknown)."""
    n = None
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            qn = max(1, int(-(-int(q) // int(per))))
            n = qn if n is None else min(n, qn)
    except (OSError, ValueError):
        pass
    return n


def cpu_thread_options(requested: int = 0):
    """Thread counts the CPU baseline is timed at: the host's cores (os.cpu_count()),
    the CPUs this process may run on (affinity mask, cgroup quota) and the OMP_NUM_THREADS the box
    sets. The best of them is reported, so a quota smaller than the core count cannot understate
    the baseline by oversubscription, nor a thread cap by under-use."""
    if requested:
        return [requested]
    n = os.cpu_count() or 1
    opts = {n}
    try:
        opts.add(len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            opts.add(max(1, int(-(-int(q) // int(per)))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        opts.add(min(int(omp), n))
    return sorted(opts, reverse=True)


def time_cpu(run_one, seconds, thread_opts, max_items=64):
    """Time `run_one()` (one unit of CPU work) at the candidate thread counts; returns (best rate,
    its threads, {threads: rate}, units, elapsed, note). Every candidate first runs the small
    warm-up unit; a count whose warm-up is over 2x the fastest one (oversubscribed: the host's
    os.cpu_count() can far exceed the CPUs this process may use) is not timed further -- one
    full-size unit there can take minutes; a count above the CPUs this process may run on is not
    even warmed up. The rest share `seconds` (at least one unit each).
    Progress goes to stderr so a long baseline is visibly alive."""
    # thread counts beyond the CPUs this process may run on (affinity mask, cgroup quota) only
    # oversubscribe them: on the GPU box os.cpu_count() is the whole host (256) against a 16-CPU
    # share, where one warm-up unit at 256 threads took minutes
    allowed = _usable_cpus()
    warm = {}
    for th in thread_opts:
        if allowed and th > allowed:
            continue
        torch.set_num_threads(th)
        run_one(warmup=True)
        t0 = time.perf_counter()
        run_one(warmup=True)
        warm[th] = time.perf_counter() - t0
        print(f"[cpu baseline] warm-up at {th} threads: {warm[th]:.3f} s", file=sys.stderr, flush=True)
    fastest = min(warm.values())
    timed = [th for th in thread_opts if th in warm and warm[th] <= 2.0 * fastest]
    skipped = {th: (warm[th] / fastest if th in warm else None) for th in thread_opts if th not in timed}
    rates, best = {}, None
    budget = seconds / len(timed)
    for th in timed:
        torch.set_num_threads(th)
        n, t0 = 0, time.perf_counter()
        while True:
            run_one(warmup=False)
            n += 1
            dt = time.perf_counter() - t0
            print(f"[cpu baseline] {th} threads: {n} unit(s) in {dt:.1f} s", file=sys.stderr, flush=True)
            if dt >= budget or n >= max_items:
                break
        rates[th] = n / dt
        if best is None or rates[th] > best[0]:
            best = (rates[th], th, n, dt)
    note = "".join(f"; {th} threads not timed (warm-up {r:.1f}x the fastest)" if r is not None else
                   f"; {th} threads not timed (more than the {allowed} CPUs this process may use)"
                   for th, r in skipped.items())
    return best[0], best[1], rates, best[2], best[3], note


def cpu_baseline_mobilenet(size, seconds, thread_opts, attention=False):
    """The CPU oracle of the MobileNet variant (fp32: the reference has no bf16 CPU path)."""
    from oracle import ref_cpu as R
    sds = []
    for m, seed in ((models.Encoder(), 5), (models.Decoder(), 6), (models.AutoEncoder().ada_out, 7)):
        sds.append(synth.live_init_(m, seed).eval().state_dict())
    kw = {}
    if attention:
        kw["att_sds"] = [synth.live_init_(models.AdaAttN(128), seed).state_dict() for seed in (8, 9)]
    c = torch.from_numpy(synth.image(821, (1, 3, size, size)))
    s = torch.from_numpy(synth.image(822, (1, 3, size, size)))

    def one(warmup):
        with torch.no_grad():
            if warmup:
                R.mb_style_transfer(c[:, :, :64, :64], s[:, :, :64, :64], *sds, **kw)
            else:
                R.mb_style_transfer(c, s, *sds, **kw)

    rate, th, rates, n, dt, note = time_cpu(one, seconds, thread_opts)
    return {"value": rate, "unit": "images/s", "cores": th, "kind": "port",
            "sample": f"{n} content+style pair(s) of 1x3x{size}x{size}, MobileNet variant, fp32 torch CPU "
                      f"({_cpu_model()}, os.cpu_count()={os.cpu_count()}), {dt:.1f} s; images/s by threads: "
                      + ", ".join(f"{k}: {v:.3f}" for k, v in rates.items()) + note}


def cpu_baseline_train(size, seconds, thread_opts):
    """The CPU oracle's AdaIN training step (oracle.ref_cpu.train_step: the same losses, backward,
    clip 2.0 + Adam on the decoder) on single image pairs."""
    from oracle import ref_cpu as R
    enc = [(torch.from_numpy(w), torch.from_numpy(b)) for w, b in synth.vgg_encoder_weights(1)]
    dec0 = [(torch.from_numpy(w), torch.from_numpy(b)) for w, b in synth.vgg_decoder_weights(2)]
    c = torch.from_numpy(synth.image(779, (1, 3, size, size)))
    s = torch.from_numpy(synth.image(780, (1, 3, size, size)))

    def one(warmup):
        dec = [(w.clone(), b.clone()) for w, b in dec0]
        if warmup:
            R.train_step(c[:, :, :64, :64], s[:, :, :64, :64], enc, dec)
        else:
            R.train_step(c, s, enc, dec)

    rate, th, rates, n, dt, note = time_cpu(one, seconds, thread_opts)
    return {"value": rate, "unit": "images/s", "cores": th, "kind": "port",
            "sample": f"{n} training step(s) on one 1x3x{size}x{size} content+style pair (AdaIN decoder, VGG loss "
                      f"network, content+style+lf+tv, clip + Adam), fp32 torch CPU ({_cpu_model()}, "
                      f"os.cpu_count()={os.cpu_count()}), {dt:.1f} s; images/s by threads: "
                      + ", ".join(f"{k}: {v:.3f}" for k, v in rates.items()) + note}


def cpu_baseline(size, seconds, thread_opts):
    """Time the CPU oracle on single 512^2 pairs (the reference's CPU path: stock torch CPU ops)."""
    from oracle import ref_cpu as R
    enc = [(torch.from_numpy(w), torch.from_numpy(b)) for w, b in synth.vgg_encoder_weights(1)[:9]]
    dec = [(torch.from_numpy(w), torch.from_numpy(b)) for w, b in synth.vgg_decoder_weights(2)]
    c = torch.from_numpy(synth.image(777, (1, 3, size, size)))
    s = torch.from_numpy(synth.image(778, (1, 3, size, size)))

    def one(warmup):
        with torch.no_grad():
            if warmup:
                R.style_transfer(c[:, :, :64, :64], s[:, :, :64, :64], enc, dec)
            else:
                R.style_transfer(c, s, enc, dec)

    rate, th, rates, n, dt, note = time_cpu(one, seconds, thread_opts)
    return {"value": rate, "unit": "images/s", "cores": th, "kind": "port",
            "sample": f"{n} content+style pair(s) of 1x3x{size}x{size}, VGG relu4_1 -> AdaIN -> decoder, "
                      f"fp32 torch CPU ({_cpu_model()}, os.cpu_count()={os.cpu_count()}), {dt:.1f} s; "
                      "images/s by threads: " + ", ".join(f"{k}: {v:.3f}" for k, v in rates.items()) + note}


def launch_ranks(args) -> int:
    """`--gpus N` without a launcher: start N rank processes of this script (one per GPU, RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run sets them) as children, wait
    for all, return the first non-zero exit code. This process never touches the GPU."""
    import signal
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    code = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                rc = p.poll()
                if rc is None:
                    continue
                pending.remove(p)
                if rc != 0 and code == 0:
                    code = rc
                    for q in pending:     # one rank failed: the others would wait forever in a collective
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return code if code >= 0 else 128 - code


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        if rank == 0:
            print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    # one process per GPU; the modulo only matters for rehearsing N ranks on a smaller box
    # (AST_BENCH_BACKEND=gloo: RCCL refuses two ranks on one device)
    local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("AST_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    if args.mode in ("train", "mobilenet", "ae-train", "ast-train"):
        {"train": train_bench, "mobilenet": mobilenet_bench, "ae-train": ae_train_bench,
         "ast-train": ast_train_bench}[args.mode](args, dev, rank, world)
        if world > 1:
            dist.destroy_process_group()
        return

    B, S = args.batch or 8, args.size or 512
    net = models.AdaINStyleTransfer().to(dev).eval()
    content = torch.from_numpy(synth.image(777 + 2 * rank, (B, 3, S, S))).to(dev)
    style = torch.from_numpy(synth.image(778 + 2 * rank, (B, 3, S, S))).to(dev)

    def step():
        with torch.no_grad():
            return net(content, style)

    for _ in range(args.warmup):
        out = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    timer = ops.LaunchTimer()
    t0 = time.perf_counter()
    with timer:
        for _ in range(args.steps):
            out = step()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], device=dev if dist.get_backend() == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert torch.isfinite(out).all(), "non-finite output"

    # ---- live roofline from the per-launch events ----
    recs = timer.results()
    conv = [(tag, fl, ms) for tag, fl, ms in recs if tag.startswith("conv3x3")]
    conv_flops = sum(fl for _, fl, _ in conv)
    conv_ms = sum(ms for _, _, ms in conv)
    n_launch = len(conv)
    avg_ms = conv_ms / n_launch
    avg_flops = conv_flops / n_launch
    achieved_tf = avg_flops / (avg_ms * 1e-3) / 1e12
    # encoder = the first 9 conv launches of every step (conv_1..conv_9 over 2B images)
    per_step = n_launch // args.steps
    enc = [r for i, r in enumerate(conv) if i % per_step < 9]
    enc_main = [r for i, r in enumerate(conv) if 1 <= i % per_step < 9]
    enc_tf = sum(f for _, f, _ in enc) / (sum(m for _, _, m in enc) * 1e-3) / 1e12
    enc_main_tf = sum(f for _, f, _ in enc_main) / (sum(m for _, _, m in enc_main) * 1e-3) / 1e12
    adain = [(tag, -fl, ms) for tag, fl, ms in recs if tag.startswith("adain")]
    adain_gbs = (sum(b for _, b, _ in adain) / (sum(m for _, _, m in adain) * 1e-3) / 1e9) if adain else None

    traffic, traffic_src = _pmc_traffic("conv_traffic.json") if (B, S) == (8, 512) else (None, None)

    images = B * world * args.steps
    result = {
        "metric": METRIC,
        "value": images / elapsed,
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (live-init VGG19/decoder weights, U[0,1) images), resident in HBM",
        "config": {"workload": f"config 2: VGG19-relu4_1 encoder (content+style) -> AdaIN -> mirrored decoder, "
                               f"bs={B}/GPU {S}x{S} fp32 forward",
                   "global_batch": B * world, "image_size": S, "parallelism": f"batch-sharded x{world}"},
        "roofline": {"bound": "mfma",
                     "kernel": "conv3x3 launches of a step (16 split-bf16 MFMA implicit-GEMM, the split-bf16 "
                               "cin <= 3 conv_1 and the direct VALU 64->3 image conv)",
                     "achieved": achieved_tf, "peak": PEAK_SPLIT_BF16_TF, "unit": "TFLOP/s",
                     "peak_basis": "fp32-accurate FLOP/s ceiling of the split-bf16 kernel = dense bf16 MFMA "
                                   "2516.6 TF / 6 bf16 products per fp32 product; achieved = algorithmic fp32 "
                                   "FLOPs / summed launch time (HIP events on the launch stream)",
                     "frac": achieved_tf / PEAK_SPLIT_BF16_TF, "traffic": traffic, "traffic_source": traffic_src,
                     "fp32_mfma_peak": PEAK_FP32_MFMA_TF, "frac_of_fp32_mfma_peak": achieved_tf / PEAK_FP32_MFMA_TF,
                     "avg_launch_ms": avg_ms, "avg_launch_gflop": avg_flops / 1e9,
                     "encoder_frac": enc_tf / PEAK_SPLIT_BF16_TF,
                     "encoder_frac_of_fp32_mfma_peak": enc_tf / PEAK_FP32_MFMA_TF,
                     "encoder_conv2_9_frac": enc_main_tf / PEAK_SPLIT_BF16_TF,
                     "adain_gbs": adain_gbs,
                     "conv_share_of_step": conv_ms / args.steps / (elapsed / args.steps * 1e3)},
    }
    if os.environ.get("BENCH_PER_LAYER"):
        layers = {}
        for i, (tag, fl, ms) in enumerate(conv):
            key = f"{i % per_step:02d} {tag}"
            a = layers.setdefault(key, [0.0, 0.0])
            a[0] += fl
            a[1] += ms
        result["per_layer"] = {k: {"ms": v[1] / args.steps, "tflops": v[0] / (v[1] * 1e-3) / 1e12}
                               for k, v in sorted(layers.items())}
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        result["cpu_baseline"] = cpu_baseline(S, args.cpu_seconds, cpu_thread_options(args.cpu_threads))
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
