"""CPU (gloo, world size 2): the data-parallel logic of dp.py — batch sharding, the flat
gradient arena and its all-reduce — driven with real decoder gradients from the CPU oracle's
AdaIN training losses. The DP step must equal the single-process step on the mean of the
per-shard losses (the DDP semantics used for BASELINE.json config 4)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from arbitrarystyletransfer_amd import dp, synth


def test_shard_range():
    assert [dp.shard_range(64, r, 8) for r in range(8)] == [(8 * r, 8 * r + 8) for r in range(8)]
    spans = [dp.shard_range(10, r, 4) for r in range(4)]
    assert spans == [(0, 3), (3, 6), (6, 8), (8, 10)]
    with pytest.raises(ValueError):   # an empty shard is refused (advisor r1)
        dp.shard_range(3, 3, 4)
    assert [dp.shard_weight(10, r, 4) for r in range(4)] == [0.3, 0.3, 0.2, 0.2]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _grads_for(content, style, lr_params):
    from oracle import ref_cpu as R
    enc = [(torch.from_numpy(w), torch.from_numpy(b)) for w, b in synth.vgg_encoder_weights(1)]
    dec = [(w.clone().requires_grad_(), b.clone().requires_grad_()) for w, b in lr_params]
    out = R.train_losses(content, style, enc, dec)
    out["loss"].backward()
    return [t.grad for wb in dec for t in wb], float(out["loss"])


def _worker(rank, world, port, content, style, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    dec_wb = [(torch.from_numpy(w), torch.from_numpy(b)) for w, b in synth.vgg_decoder_weights(2)]
    a, b = dp.shard_range(content.shape[0], rank, world)
    grads, loss = _grads_for(content[a:b], style[a:b], dec_wb)
    params = [torch.nn.Parameter(t.clone()) for wb in dec_wb for t in wb]
    for p, g in zip(params, grads):
        p.grad = g
    arena = dp.FlatGradArena(params, device=torch.device("cpu"))
    try:
        arena.all_reduce()
    finally:
        arena.unregister()
    if rank == 0:
        torch.save({"flat": arena.flat.clone(), "loss": loss}, result_path)
    dist.barrier()
    dist.destroy_process_group()


def test_dp_gradient_average_matches_single_process(tmp_path):
    content = torch.from_numpy(synth.image(901, (4, 3, 16, 16)))
    style = torch.from_numpy(synth.image(902, (4, 3, 16, 16)))
    path = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(2, _free_port(), content, style, path), nprocs=2, join=True)
    got = torch.load(path, weights_only=True)["flat"]
    dec_wb = [(torch.from_numpy(w), torch.from_numpy(b)) for w, b in synth.vgg_decoder_weights(2)]
    g0, _ = _grads_for(content[:2], style[:2], dec_wb)
    g1, _ = _grads_for(content[2:], style[2:], dec_wb)
    ref = torch.cat([((x + y) / 2).reshape(-1) for x, y in zip(g0, g1)])
    np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=1e-5, atol=1e-7 * float(ref.abs().max()))


def _style_worker(rank, world, port, content, style, result_path):
    """One style (owned by rank 0), contents sharded: rank 0 broadcasts relu4_1 style stats."""
    from oracle import ref_cpu as R
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    enc = [(torch.from_numpy(w), torch.from_numpy(b)) for w, b in synth.vgg_encoder_weights(1)[:9]]
    dec = [(torch.from_numpy(w), torch.from_numpy(b)) for w, b in synth.vgg_decoder_weights(2)]
    with torch.no_grad():
        if rank == 0:
            m, s = R.channel_stats(R.vgg_encoder(style, enc)[0])
            m, s = m.flatten(), s.flatten()
        else:
            m, s = torch.zeros(512), torch.full((512,), float("nan"))
        m, s = dp.broadcast_style_stats(m, s, src=0)
        a, b = dp.shard_range(content.shape[0], rank, world)
        t = R.adain_from_stats(R.vgg_encoder(content[a:b], enc)[0], m, s)
        y = R.vgg_decoder(t, dec)
    torch.save({"m": m, "s": s, "y": y}, result_path + f".{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_style_stats_broadcast_one_style_many_contents(tmp_path):
    from oracle import ref_cpu as R
    content = torch.from_numpy(synth.image(911, (4, 3, 32, 32)))
    style = torch.from_numpy(synth.image(912, (1, 3, 32, 32)))
    path = str(tmp_path / "st")
    mp.spawn(_style_worker, args=(2, _free_port(), content, style, path), nprocs=2, join=True)
    r0 = torch.load(path + ".0", weights_only=True)
    r1 = torch.load(path + ".1", weights_only=True)
    assert torch.equal(r0["m"], r1["m"]) and torch.equal(r0["s"], r1["s"])
    enc = [(torch.from_numpy(w), torch.from_numpy(b)) for w, b in synth.vgg_encoder_weights(1)[:9]]
    dec = [(torch.from_numpy(w), torch.from_numpy(b)) for w, b in synth.vgg_decoder_weights(2)]
    with torch.no_grad():
        ref = R.style_transfer(content, style.expand(4, -1, -1, -1), enc, dec)
    got = torch.cat([r0["y"], r1["y"]])
    # CPU convs on different batch sizes pick different algorithms: fp32 reassociation only
    np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=1e-4, atol=1e-4 * float(np.nanmax(np.abs(ref.numpy()))))


def _syncbn_worker(rank, world, port, x, result_path):
    """SyncBatchNorm plumbing (dp.py): per-rank (count, mean, M2) gathered over gloo and merged
    (oracle Chan merge) equal the whole batch's statistics; the backward sums all-reduce."""
    from oracle import ref_cpu as R
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b = dp.shard_range(x.shape[0], rank, world)
    local = torch.from_numpy(R.bn_shard_stats(x[a:b].numpy()))
    allst = dp.all_gather_bn_stats(local)
    sums = torch.tensor([[float(rank + 1)] * 3, [2.0 * (rank + 1)] * 3])
    dp.all_reduce_sum(sums)
    bn = torch.nn.BatchNorm2d(3)
    assert dp.sync_group(bn) is None
    dp.convert_sync_batchnorm(torch.nn.Sequential(bn))
    assert dp.sync_group(bn) is not None
    torch.save({"allst": allst, "sums": sums}, result_path + f".{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_syncbn_stats_gather_and_merge(tmp_path):
    from oracle import ref_cpu as R
    x = torch.from_numpy(synth.image(931, (5, 3, 7, 6))) * 3 + 2   # ragged shards: 3 + 2 images
    path = str(tmp_path / "bn")
    mp.spawn(_syncbn_worker, args=(2, _free_port(), x, path), nprocs=2, join=True)
    r0 = torch.load(path + ".0", weights_only=True)
    r1 = torch.load(path + ".1", weights_only=True)
    assert torch.equal(r0["allst"], r1["allst"]) and r0["allst"].shape == (2, 3, 3)
    mu, var, cnt = R.bn_merge_stats(r0["allst"].numpy())
    xn = x.numpy().astype(np.float64)
    np.testing.assert_allclose(mu, xn.mean(axis=(0, 2, 3)), rtol=1e-12)
    np.testing.assert_allclose(var, xn.var(axis=(0, 2, 3)), rtol=1e-10)
    assert (cnt == 5 * 7 * 6).all()
    assert torch.equal(r0["sums"], torch.tensor([[3.0] * 3, [6.0] * 3])) and torch.equal(r0["sums"], r1["sums"])


def _world8_worker(rank, world, port, content, style, result_path):
    """BASELINE.json config 4's data-parallel step at world size 8 (gloo): AdaINTrainer's semantics
    (arbitrarystyletransfer_amd/train.py:202-215) with the oracle's losses — each rank weights its
    batch-mean terms by local/global (the sum-type TV term is additive), backward, the flat arena's
    SUM all-reduce, clip_grad_norm_(2.0) + Adam (train.py:287-300). Also the one-style broadcast and
    an 8-part SyncBatchNorm gather + merge."""
    from oracle import ref_cpu as R
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    gb = content.shape[0]
    a, b = dp.shard_range(gb, rank, world)
    w = dp.shard_weight(gb, rank, world)
    enc = [(torch.from_numpy(x), torch.from_numpy(y)) for x, y in synth.vgg_encoder_weights(1)]
    dec = [(torch.from_numpy(x).clone().requires_grad_(), torch.from_numpy(y).clone().requires_grad_())
           for x, y in synth.vgg_decoder_weights(2)]
    params = [p for wb in dec for p in wb]
    out = R.train_losses(content[a:b], style[a:b], enc, dec)
    (w * (1.25 * out["content_loss"] + 0.5 * out["style_loss"] + 1.0 * out["lf_loss"])
     + 0.0006 * out["tv_loss"]).backward()
    arena = dp.FlatGradArena(params, device=torch.device("cpu"), average=False)
    try:
        arena.all_reduce()
    finally:
        arena.unregister()
    grads = [p.grad.detach().clone() for p in params]
    opt = torch.optim.Adam(params, lr=2e-4, betas=[0.9, 0.999], eps=1e-5)
    norm = torch.nn.utils.clip_grad_norm_(params, 2.0, error_if_nonfinite=True)
    opt.step()
    # one style image owned by rank 0, broadcast to every rank
    with torch.no_grad():
        if rank == 0:
            m, s = R.channel_stats(R.vgg_encoder(style[:1], enc[:9])[0])
            m, s = m.flatten(), s.flatten()
        else:
            m, s = torch.zeros(512), torch.full((512,), float("nan"))
        m, s = dp.broadcast_style_stats(m, s, src=0)
    # SyncBatchNorm statistics of an 8-way sharded activation
    act = content[:, :, :5, :7] * 3 + 1
    allst = dp.all_gather_bn_stats(torch.from_numpy(R.bn_shard_stats(act[a:b].numpy())))
    torch.save({"grads": grads, "params": [p.detach().clone() for p in params], "norm": float(norm),
                "m": m, "s": s, "allst": allst}, result_path + f".{rank}")
    dist.barrier()
    dist.destroy_process_group()


def _shard_grads(content, style, a, b, w, dtype):
    """Decoder gradients of AdaINTrainer's rank-local objective on images a..b (shard weight w)."""
    from oracle import ref_cpu as R
    enc = [(torch.from_numpy(x).to(dtype), torch.from_numpy(y).to(dtype)) for x, y in synth.vgg_encoder_weights(1)]
    dec = [(torch.from_numpy(x).to(dtype).requires_grad_(), torch.from_numpy(y).to(dtype).requires_grad_())
           for x, y in synth.vgg_decoder_weights(2)]
    out = R.train_losses(content[a:b].to(dtype), style[a:b].to(dtype), enc, dec)
    (w * (1.25 * out["content_loss"] + 0.5 * out["style_loss"] + 1.0 * out["lf_loss"])
     + 0.0006 * out["tv_loss"]).backward()
    return [p.grad for wb in dec for p in wb]


def test_dp_world8_step_matches_single_process(tmp_path):
    """Config 4 readiness without an 8-GPU node: 8 gloo ranks, a global batch
    of 13 (uneven shards 2,2,2,2,2,1,1,1). (1) The semantics, in float64: the shard-weighted rank
    objectives sum to exactly the single-process full-batch gradient. (2) The plumbing, in fp32: the
    arena's SUM all-reduce equals the rank gradients summed here, every rank holds the same reduced
    gradient, gradient norm and post-clip + Adam weights (equal to torch's clip + Adam on that sum),
    the same broadcast style statistics, and the same 8-part BatchNorm statistics, whose merge equals
    the whole batch's. (fp32 is not compared with the full-batch step itself: the oracle's fp32
    evaluation moves by ~1e-2 relative between batch sizes through the 2x2 mean-variance-norm taps,
    while float64 agrees to 1e-13.)"""
    from oracle import ref_cpu as R
    gb, world = 13, 8
    spans = [dp.shard_range(gb, r, world) for r in range(world)]
    assert [b - a for a, b in spans] == [2, 2, 2, 2, 2, 1, 1, 1]
    content = torch.from_numpy(synth.image(951, (gb, 3, 32, 32)))
    style = torch.from_numpy(synth.image(952, (gb, 3, 32, 32)))
    # (1) semantics
    full = _shard_grads(content, style, 0, gb, 1.0, torch.float64)
    parts = [_shard_grads(content, style, a, b, dp.shard_weight(gb, r, world), torch.float64)
             for r, (a, b) in enumerate(spans)]
    for i, g in enumerate(full):
        s = sum(p[i] for p in parts)
        assert float((s - g).abs().max()) <= 1e-10 * float(g.abs().max()), i
    # (2) plumbing
    path = str(tmp_path / "w8")
    mp.spawn(_world8_worker, args=(world, _free_port(), content, style, path), nprocs=world, join=True)
    res = [torch.load(path + f".{r}", weights_only=True) for r in range(world)]
    for r in range(world):
        for g0, g in zip(res[0]["grads"], res[r]["grads"]):
            assert torch.equal(g0, g)
        for p0, p in zip(res[0]["params"], res[r]["params"]):
            assert torch.equal(p0, p)
        assert torch.equal(res[r]["m"], res[0]["m"]) and torch.equal(res[r]["s"], res[0]["s"])
        assert torch.equal(res[r]["allst"], res[0]["allst"])
    nt = torch.get_num_threads()
    torch.set_num_threads(1)   # as the ranks: the oracle's fp32 gradients depend on the CPU kernels' split
    try:
        parts32 = [_shard_grads(content, style, a, b, dp.shard_weight(gb, r, world), torch.float32)
                   for r, (a, b) in enumerate(spans)]
    finally:
        torch.set_num_threads(nt)
    ref = [sum(p[i] for p in parts32) for i in range(len(parts32[0]))]
    for g, gr in zip(res[0]["grads"], ref):   # the collective's summation order only
        np.testing.assert_allclose(g.numpy(), gr.numpy(), rtol=1e-5, atol=1e-6 * float(gr.abs().max()))
    params = [torch.nn.Parameter(torch.from_numpy(x).clone()) for wb in synth.vgg_decoder_weights(2) for x in wb]
    for p, g in zip(params, ref):
        p.grad = g.clone()
    opt = torch.optim.Adam(params, lr=2e-4, betas=[0.9, 0.999], eps=1e-5)
    norm = torch.nn.utils.clip_grad_norm_(params, 2.0, error_if_nonfinite=True)
    opt.step()
    np.testing.assert_allclose(res[0]["norm"], float(norm), rtol=1e-5)
    for p, pr in zip(res[0]["params"], params):
        diff = (p - pr.detach()).abs()
        # Adam's first step is ~lr*sign(g): elements whose gradient is within rounding of 0 may differ
        assert float((diff > 1e-6).float().mean()) <= 1e-3 and float(diff.max()) <= 4e-4
    enc = [(torch.from_numpy(x), torch.from_numpy(y)) for x, y in synth.vgg_encoder_weights(1)]
    with torch.no_grad():
        m, s = R.channel_stats(R.vgg_encoder(style[:1], enc[:9])[0])
    np.testing.assert_allclose(res[0]["m"].numpy(), m.flatten().numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(res[0]["s"].numpy(), s.flatten().numpy(), rtol=1e-5, atol=1e-6)
    assert res[0]["allst"].shape == (world, 3, 3)
    mu, var, cnt = R.bn_merge_stats(res[0]["allst"].numpy())
    act = (content[:, :, :5, :7] * 3 + 1).numpy().astype(np.float64)
    np.testing.assert_allclose(mu, act.mean(axis=(0, 2, 3)), rtol=1e-10)
    np.testing.assert_allclose(var, act.var(axis=(0, 2, 3)), rtol=1e-9)
    assert (cnt == gb * 5 * 7).all()
