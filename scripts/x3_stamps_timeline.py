#!/usr/bin/env python3
"""Per-workgroup timeline of conv3x3_x3_kernel stamp records (scripts/x3_stamps.py):
python scripts/x3_stamps_timeline.py FILE.npz [FILE2.npz ...]. Chunk period = one barrier-2 release
to the next; MFMA window = the first wave's MFMA start to the first / last wave's MFMA end; store
window = barrier-1 release to barrier-2 release (all in shader cycles, means over workgroups)."""
import sys

import numpy as np


def timeline(path):
    rec = np.load(path)["rec"]
    valid = rec[:, :, 196] == 0x57a3
    nch = int(rec[valid][0, 195])
    W = rec[:, :8, :4 + 4 * nch].astype(np.int64)[valid[:, :8].all(1)]
    T = (W - W[:, :, :1].min(1, keepdims=True)) % (1 << 32)
    b2 = [T[:, :, 1].max(1)] + [T[:, :, 5 + 4 * k].max(1) for k in range(nch - 1)]
    cyc = np.diff(np.stack(b2, 1), axis=1)
    first = np.stack([T[:, :, 3 + 4 * k].min(1) - T[:, :, 2 + 4 * k].min(1) for k in range(nch - 1)], 1)
    last = np.stack([T[:, :, 3 + 4 * k].max(1) - T[:, :, 2 + 4 * k].min(1) for k in range(nch - 1)], 1)
    b1 = np.stack([T[:, :, 4 + 4 * k].max(1) - T[:, :, 3 + 4 * k].max(1) for k in range(nch - 1)], 1)
    sw = np.stack([T[:, :, 5 + 4 * k].max(1) - T[:, :, 4 + 4 * k].max(1) for k in range(nch - 1)], 1)
    end = T[:, :, 3 + 4 * nch].max(1)
    print(f"{path}: {len(T)} workgroups, {nch} chunks; workgroup {end.mean():.0f} cycles; prologue "
          f"{T[:, :, 1].max(1).mean():.0f}; chunk period {cyc.mean():.0f}; MFMA window to first / last wave done "
          f"{first.mean():.0f} / {last.mean():.0f}; last wave -> barrier-1 release {b1.mean():.0f}; store window "
          f"{sw.mean():.0f}; epilogue {(end - T[:, :, 2 + 4 * nch].max(1)).mean():.0f}")


def steps(path, chunk=5, nstep=18):
    """Per-step timeline of one chunk (X3_STAMP build: stamps 4 + 4 nch + step of chunk 5), for the
    two waves of each SIMD pair (waves w and w + 4): mean start of each step relative to the chunk's
    first MFMA-phase stamp, and the MFMA-phase end."""
    rec = np.load(path)["rec"]
    valid = rec[:, :, 196] == 0x57a3
    nch = int(rec[valid][0, 195])
    W = rec[:, :8, :4 + 4 * nch + nstep].astype(np.int64)[valid[:, :8].all(1)]
    t0 = W[:, :, 2 + 4 * chunk].min(1, keepdims=True)
    S = (W[:, :, 4 + 4 * nch:4 + 4 * nch + nstep] - t0[:, :, None]) % (1 << 32)
    end = (W[:, :, 3 + 4 * chunk] - t0) % (1 << 32)
    a, b = S[:, :4], S[:, 4:]                       # waves w and w + 4 of each pair
    ea, eb = end[:, :4], end[:, 4:]
    sel = (ea <= eb)[:, :, None]
    firstw = np.where(sel, a, b).reshape(-1, nstep)   # the pair's first-finishing wave
    lastw = np.where(sel, b, a).reshape(-1, nstep)
    print("  first-finishing wave of a pair: step starts", np.round(firstw.mean(0)).astype(int).tolist())
    print("  last-finishing wave of a pair:  step starts", np.round(lastw.mean(0)).astype(int).tolist())
    older = (ea <= eb).mean()
    print(f"  the older wave (w < 4) finishes first in {older:.0%} of pairs")
    print("  MFMA-phase ends (first / last of a pair):", int(np.minimum(end[:, :4], end[:, 4:]).mean()),
          int(np.maximum(end[:, :4], end[:, 4:]).mean()))


if __name__ == "__main__":
    for p in sys.argv[1:]:
        timeline(p)
        try:
            steps(p)
        except (IndexError, ValueError):
            pass
