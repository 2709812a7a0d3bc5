"""The RCCL branches of dp.py executed on one GPU: a fresh child process
(tests/rccl_ws1_worker.py) initialises torch.distributed "nccl" (= RCCL on ROCm) at world size 1
with device_id and runs the trainers' data-parallel path -- the FlatGradArena all-reduce in SUM and
AVG modes, SyncBatchNorm's all_gather_into_tensor and all-reduce, the style-statistics broadcast --
against the same computation without a process group (bitwise; bound 1e-6 relative).

8-rank RCCL over xGMI (configs 4 and the scaling curve) is run by the driver's multi-GPU bench, not
here: one box has one GPU, and RCCL refuses two ranks on one device.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def test_rccl_world1_matches_single_process(tmp_path):
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    out = tmp_path / "rccl.json"
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rccl_ws1_worker.py")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    r = subprocess.run([sys.executable, worker, str(out)], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rep = json.loads(out.read_text())
    print(json.dumps(rep))
    for k in ("adain_trainer_sum", "arena_avg", "ae_syncbn_step", "broadcast_style_stats"):
        assert rep[k]["rel_inf"] <= 1e-6, (k, rep[k])
    assert rep["adain_trainer_sum"]["bitwise"] and rep["arena_avg"]["bitwise"]
