"""Diff maps of the run-to-run variation under concurrent GPU load.

The layer walk of race_probe3.py (VGG encoder over content + style, every conv3x3 launch kept),
repeated N times against the first walk; for every repeat whose outputs differ, the FIRST differing
launch is described: how many elements differ, by how much, in which images / channels / rows /
columns, and which kernel tiles they fall in (the direct cin<=4 kernel's TH x 128-pixel tiles, the
split-bf16 kernel's 16 x 32-pixel x 64-channel tiles). Then the same launch is re-run 4 times on the
same (reference) inputs. Tile-aligned blocks point at one workgroup's LDS or registers, scattered
elements at stale reads, all-element rounding-level changes at a changed input or code path.
Also checks that the walk's inputs and packed weights are unchanged after every repeat.
Writes the masks of the first two differing launches to <out>/race_probe4_<k>.npz."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from arbitrarystyletransfer_amd import models, ops, synth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 16
OUT = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
dev = torch.device("cuda")


def rnd(seed, shape):
    return torch.from_numpy(synth.uniform(seed, int(np.prod(shape))).astype(np.float32).reshape(shape)).to(dev)


net = models.AdaINStyleTransfer().to(dev)
enc = net.encoder
c, s = rnd(16, (2, 3, 128, 96)), rnd(17, (2, 3, 128, 96))
c0, s0 = c.clone(), s.clone()
norm = enc._vgg_layers[0]


def launch(idx, conv, cur, cur2, want_pre, want_act, want_pool):
    first = idx == 1
    return ops.conv3x3(cur, enc._packed.get(conv), conv.bias, conv.out_channels, pad_mode="zeros",
                       in_mean=norm.mean.view(-1) if first else None,
                       in_std=norm.std.view(-1) if first else None,
                       want_pre=want_pre, want_act=want_act, want_pool=want_pool, x2=cur2)


def walk():
    res = []
    cur, cur2 = c, s
    for idx, conv, want_pre, want_act, want_pool, collect in enc._plan():
        outs = launch(idx, conv, cur, cur2, want_pre, want_act, want_pool)
        n, cin, h, w = cur.shape[0] + (cur2.shape[0] if cur2 is not None else 0), cur.shape[1], cur.shape[2], cur.shape[3]
        cfg = ops.tuned_config(n, cin, h, w, conv.out_channels, 1, "zeros", want_pool)
        G, _ = ops.pack_plan(n, w, want_pool)
        tag = f"conv_{idx} {cin}->{conv.out_channels} {h}x{w} n{n} pool{want_pool} cfg{cfg} G{G}"
        inp = (cur.clone(), cur2.clone() if cur2 is not None else None)
        res.append((tag, [t.clone() for t in outs if t is not None], (idx, conv, want_pre, want_act, want_pool), inp))
        cur, cur2 = (outs[2] if want_pool else outs[1]), None
    return res


def same(a, b):
    return torch.equal(a, b) or bool(((a == b) | (torch.isnan(a) & torch.isnan(b))).all())


def describe(name, got, ref, th):
    mask = got != ref
    mask &= ~(torch.isnan(got) & torch.isnan(ref))
    nd = int(mask.sum())
    d = (got - ref).abs()[mask]
    r = ref.abs()[mask]
    print(f"   {name} {tuple(ref.shape)}: {nd} of {ref.numel()} elements differ; max|d| {float(d.max()):.3e} "
          f"(max|ref| {float(ref.abs().max()):.3e}); median |d|/|ref| {float((d / r.clamp_min(1e-30)).median()):.3e}",
          flush=True)
    idx = mask.nonzero().cpu().numpy()
    n_, co, y, x = idx[:, 0], idx[:, 1], idx[:, 2], idx[:, 3]
    print(f"     images {sorted(set(n_.tolist()))}; channels {len(set(co.tolist()))} of {ref.shape[1]} "
          f"(min {co.min()}, max {co.max()}); rows {y.min()}..{y.max()}; cols {x.min()}..{x.max()}", flush=True)
    for tag, tr, tc, tco in ((f"direct TH{th}x128", th, 128, ref.shape[1]), ("x3 16x32x64", 16, 32, 64)):
        tiles = {}
        for a, b, e, f in zip(n_.tolist(), co.tolist(), y.tolist(), x.tolist()):
            key = (a, b // tco, e // tr, f // tc)
            tiles[key] = tiles.get(key, 0) + 1
        full = tr * tc * min(tco, ref.shape[1])
        top = sorted(tiles.items(), key=lambda kv: -kv[1])[:6]
        print(f"     {tag} tiles touched: {len(tiles)}; largest {[(k, v, round(v / full, 3)) for k, v in top]}",
              flush=True)
    return mask


def conv1_terms(conv, n_, co, y, x):
    """The 27 products of conv_1's FMA chain at (n, co, y, x), in the kernel's order (tap-major,
    channel-minor), on the CPU from the normalised, zero-padded input."""
    xin = torch.cat([c, s]).cpu()
    xn = (xin - norm.mean.cpu().view(1, -1, 1, 1)) / norm.std.cpu().view(1, -1, 1, 1)
    xp = torch.nn.functional.pad(xn, (1, 1, 1, 1))
    w = conv.weight.detach().cpu()
    t = torch.empty(27, dtype=torch.float64)
    for ky in range(3):
        for kx in range(3):
            for ch in range(3):
                t[(ky * 3 + kx) * 3 + ch] = float(xp[n_, ch, y + ky, x + kx]) * float(w[co, ch, ky, kx])
    return t


def explain_conv1(conv, got, ref, mask):
    """Is got - ref exactly a contiguous run of the FMA chain's products (skipped or repeated
    instructions), or something else (a foreign value)?"""
    idx = mask.nonzero().cpu().numpy()
    g, r = got.cpu(), ref.cpu()
    kinds = {}
    for k, (a, b, e, f) in enumerate(idx[:80]):
        d = float(g[a, b, e, f]) - float(r[a, b, e, f])
        if float(g[a, b, e, f]) == 0.0 or float(r[a, b, e, f]) == 0.0:
            kinds["relu-clipped"] = kinds.get("relu-clipped", 0) + 1
            continue
        t = conv1_terms(conv, a, b, e, f)
        pre = torch.cat([torch.zeros(1, dtype=torch.float64), torch.cumsum(t, 0)])
        best = (abs(d), None)
        for i in range(27):
            for j in range(i + 1, 28):
                run = float(pre[j] - pre[i])
                for sgn, lab in ((-1, "missing"), (1, "doubled")):
                    err = abs(d - sgn * run)
                    if err < best[0]:
                        best = (err, f"{lab} products {i}..{j - 1}")
        tol = 1e-5 * max(1.0, abs(float(r[a, b, e, f])))
        kind = best[1] if best[0] <= tol else "no product run"
        kinds[kind.split(' products')[0] if best[0] <= tol else kind] = kinds.get(
            kind.split(' products')[0] if best[0] <= tol else kind, 0) + 1
        if k < 12:
            print(f"     ({a},{b},{e},{f}) got {float(g[a, b, e, f]):.6g} ref {float(r[a, b, e, f]):.6g} d {d:.6g}: "
                  f"{kind} (residual {best[0]:.2e})", flush=True)
    print(f"     explanation counts over {min(80, len(idx))} elements: {kinds}", flush=True)


with torch.no_grad():
    ref = walk()
    pk_ref = [enc._packed.get(conv).clone() for _, _, (idx, conv, *_), _ in ref]
    saved = 0
    bad_total = 0
    for rep in range(N):
        got = walk()
        first = None
        for i, ((tag, a, _, _), (_, b, _, _)) in enumerate(zip(got, ref)):
            if any(not same(x, y) for x, y in zip(a, b)):
                first = i
                break
        ins_ok = same(c, c0) and same(s, s0)
        pk_ok = all(same(enc._packed.get(conv), p) for (_, _, (idx, conv, *_), _), p in zip(ref, pk_ref))
        if first is None:
            print(f"repeat {rep}: same (inputs unchanged {ins_ok}, packed weights unchanged {pk_ok})", flush=True)
            continue
        bad_total += 1
        tag = got[first][0]
        print(f"repeat {rep}: FIRST DIFFERING LAUNCH {tag} (inputs unchanged {ins_ok}, packed weights unchanged {pk_ok})",
              flush=True)
        th = 8 if first == 0 else 16
        inp_same = all((x is None and y is None) or same(x, y) for x, y in zip(got[first][3], ref[first][3]))
        print(f"   launch inputs equal to the reference walk's: {inp_same}", flush=True)
        masks = []
        for k, (x, y) in enumerate(zip(got[first][1], ref[first][1])):
            if not same(x, y):
                m = describe(f"output {k}", x, y, th)
                if first == 0:
                    explain_conv1(got[first][2][1], x, y, m)
                masks.append(m.cpu().numpy())
        # re-run the same launch on the reference walk's inputs
        idx, conv, wp_, wa_, wpo_ = ref[first][2]
        rin = ref[first][3]
        for t in range(4):
            outs = [o for o in launch(idx, conv, rin[0], rin[1], wp_, wa_, wpo_) if o is not None]
            eq_ref = all(same(o, y) for o, y in zip(outs, ref[first][1]))
            eq_got = all(same(o, y) for o, y in zip(outs, got[first][1]))
            print(f"   re-run {t}: equals reference {eq_ref}, equals the differing result {eq_got}", flush=True)
        if saved < 2:
            os.makedirs(OUT, exist_ok=True)
            np.savez_compressed(os.path.join(OUT, f"race_probe4_{saved}.npz"),
                                **{f"mask{k}": np.packbits(m) for k, m in enumerate(masks)},
                                **{f"shape{k}": np.array(m.shape) for k, m in enumerate(masks)})
            saved += 1
    torch.cuda.synchronize()
print(f"{bad_total} of {N} repeats differ", flush=True)
