#!/usr/bin/env python3
"""Summary of conv3x3_x3_kernel stamp records (scripts/x3_stamps.py). python scripts/x3_stamps_summary.py FILE.npz"""
import sys

import numpy as np

MFMA_PER_CHUNK = 432  # tile 28 (8 waves, 2 rows x 32 px x 64 ch per wave): 9 taps x 2 rows x 2 x 4 x 3
MFMA_CYC = 16         # v_mfma_f32_16x16x32_bf16 issue cycles on one SIMD


def summary(rec):
    valid = rec[:, :, 196] == 0x57a3
    waves = rec[valid]
    if len(waves) == 0:
        print("no records")
        return
    nch = int(waves[0, 195])
    st = waves[:, :4 + 4 * nch].astype(np.int64)
    d = lambda a, b: (st[:, b] - st[:, a]) % (1 << 32)  # noqa: E731
    total = d(0, 3 + 4 * nch)
    pro = d(0, 1)
    mf = np.stack([d(2 + 4 * k, 3 + 4 * k) for k in range(nch)], 1)
    issue = np.stack([d(1 if k == 0 else 5 + 4 * (k - 1), 2 + 4 * k) for k in range(nch)], 1)
    b1 = np.stack([d(3 + 4 * k, 4 + 4 * k) for k in range(nch - 1)], 1) if nch > 1 else np.zeros((len(st), 0))
    sto = np.stack([d(4 + 4 * k, 5 + 4 * k) for k in range(nch - 1)], 1) if nch > 1 else np.zeros((len(st), 0))
    epi = d(2 + 4 * nch, 3 + 4 * nch)
    tail = d(3 + 4 * (nch - 1), 2 + 4 * nch)
    print(f"{len(st)} waves, {nch} K chunks; cycles per wave (median over waves):")
    med = lambda v: float(np.median(v))  # noqa: E731
    parts = {"prologue (chunk-0 gather+split+store, barrier)": pro.astype(float),
             "load issue (next chunk's buffer loads)": issue.sum(1).astype(float),
             "MFMA phases": mf.sum(1).astype(float),
             "barrier 1 wait (after MFMAs)": b1.sum(1).astype(float),
             "store phase (split + LDS writes + barrier 2)": sto.sum(1).astype(float),
             "last-chunk tail to epilogue": tail.astype(float),
             "epilogue (staged stores, to vmcnt 0)": epi.astype(float)}
    tot = med(total)
    for k, v in parts.items():
        print(f"  {k:48s} {med(v):9.0f}  {med(v) / tot:6.1%}")
    print(f"  {'total':48s} {tot:9.0f}")
    print(f"  per chunk: MFMA phase median {med(mf):.0f} cycles (alone on a SIMD: {MFMA_PER_CHUNK * MFMA_CYC}, "
          f"two waves sharing the pipe: {2 * MFMA_PER_CHUNK * MFMA_CYC}); barrier-1 wait {med(b1) if b1.size else 0:.0f}; "
          f"store phase {med(sto) if sto.size else 0:.0f}")
    # SIMD partners: waves of one workgroup with equal SIMD id (HW_ID bits 5:4)
    hw = waves[:, 192]
    simd = (hw >> 4) & 3
    print(f"  SIMD ids of workgroup 0's waves: {list(simd[:8])}")


if __name__ == "__main__":
    summary(np.load(sys.argv[1])["rec"])
