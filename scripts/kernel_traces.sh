#!/bin/bash
# rocprofv3 --kernel-trace --stats of bench modes at the current tree (GPU box):
#   bash scripts/kernel_traces.sh TAG MODE [MODE ...]   -> gpurun_out/TAG/ks_MODE/..., ks_MODE.json
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for mode in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ks_$mode" -o ks \
      -- python3 "$R/bench.py" --mode "$mode" --steps 10 --warmup 3 --cpu-seconds 0 > "$O/ks_$mode.json" 2> "$O/ks_$mode.err" \
    || { echo "kernel trace $mode failed"; exit 1; }
  echo "kernel trace $mode ok: $(cut -c1-200 "$O/ks_$mode.json")"
done
