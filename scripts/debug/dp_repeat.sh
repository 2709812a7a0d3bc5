#!/bin/bash
# run the 2-rank AE / AST DP workers 3 times each and report which saved tensors differ run to run
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"; OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
for w in ${DP_WORKERS:-ae ast}; do
  for i in 1 2 3; do
    timeout -k 10 150 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
      --master-port=$((29600 + i)) tests/${w}_dp_worker.py $OUT/dp_${w}_$i.npz > $OUT/dp_${w}_$i.log 2>&1 || { tail -5 $OUT/dp_${w}_$i.log; exit 1; }
  done
done
python3 - <<'PY'
import numpy as np, os
out = os.environ.get("GRAFT_REPO_ROOT", ".") + "/gpurun_out"
for w in os.environ.get("DP_WORKERS", "ae ast").split():
    r = [np.load(f"{out}/dp_{w}_{i}.npz") for i in (1, 2, 3)]
    diff = []
    for k in r[0].files:
        for o in r[1:]:
            if not np.array_equal(r[0][k], o[k]):
                a, b = r[0][k], o[k]
                diff.append((float(np.abs(a - b).max() / max(np.abs(a).max(), 1e-30)), k))
                break
    diff.sort(reverse=True)
    print(w, len(r[0].files), "tensors;", len(diff), "differ;", diff[:8])
    for kind in ("grad:", "param:", "buf:"):
        dk = [d for d in diff if d[1].startswith(kind)]
        print("  ", kind, len(dk), "differ; smallest", sorted(dk)[:4])
for i in (1, 2, 3):
    for w in os.environ.get("DP_WORKERS", "ae ast").split():
        os.remove(f"{out}/dp_{w}_{i}.npz")
PY
