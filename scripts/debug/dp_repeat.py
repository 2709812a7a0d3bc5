"""Runs tests/ae_dp_worker.py (2 gloo ranks on the one GPU) several times and reports, per run, the
largest relative gradient error against the golden file and whether each run's outputs are
bit-identical to the first run's. Used to tell run-to-run nondeterminism from a fixed numerical gap."""
import os
import socket
import subprocess
import sys

import numpy as np

root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
worker = os.path.join(root, "tests", "ae_dp_worker.py")
golden = np.load(os.path.join(root, "tests", "golden", "ae_train_step_64.npz"))
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 4
outdir = sys.argv[2] if len(sys.argv) > 2 else "/tmp"
nproc = int(os.environ.get("DP_NPROC", "2"))   # AST_POISON in the environment reaches the worker
first = None
for it in range(runs):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = os.path.join(outdir, f"dp_{it}.npz")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
                        "--master-addr=127.0.0.1", f"--master-port={port}", worker, out],
                       capture_output=True, text=True, timeout=240)
    if r.returncode != 0:
        print(r.stdout[-2000:], r.stderr[-2000:])
        sys.exit(1)
    got = dict(np.load(out))
    import hashlib
    h = hashlib.sha1(b"".join(np.ascontiguousarray(got[k]).tobytes() for k in sorted(got) if k.startswith("grad:")))
    print(f"run {it}: CUs {got.pop('cus', '?')} arch {got.pop('gcn', '?')} grad sha1 {h.hexdigest()[:16]}", flush=True)
    norm = float(got["grad_norm"])
    worst, wk = 0.0, None
    for key in golden.files:
        if not key.startswith("grad:"):
            continue
        ref = golden[key]
        mine = got[key].reshape(-1)
        mine = (mine if mine.size == ref.size else mine[::17]).reshape(ref.shape)
        e = float(np.abs(mine - ref).max()) / max(float(np.abs(ref).max()), 1e-5 * norm)
        if e > worst:
            worst, wk = e, key
    diff = []
    if first is None:
        first = got
    else:
        diff = [k for k in got if not np.array_equal(got[k], first[k])]
    print(f"run {it}: worst {worst:.3e} ({wk}); keys differing from run 0: {len(diff)} {diff[:6]}", flush=True)
    for k in diff[:40]:
        a, b = np.asarray(got[k], np.float64), np.asarray(first[k], np.float64)
        d = np.abs(a - b)
        print(f"   {k} shape {a.shape}: max|d| {d.max():.3e} rel {d.max() / max(np.abs(b).max(), 1e-30):.3e} "
              f"elements differing {int((d > 0).sum())}/{d.size} first at {np.unravel_index(int(np.argmax(d > 0)), d.shape)}",
              flush=True)
