#!/bin/bash
# Profiles behind the bench's roofline fields, at the current tree (run on the GPU box):
#   rocprofv3 --kernel-trace --stats of each bench mode, and FETCH_SIZE / WRITE_SIZE passes (one
#   counter per run, no trace domains) for config 2 (conv3x3) and config 5 (mb expand_dw).
# Then, here: python scripts/pmc_traffic.py <tag>/tr_fwd conv3x3 profiles/conv_traffic.json (etc.)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r02m}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for mode in fwd train mobilenet; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ks_$mode" -o ks \
      -- python3 "$R/bench.py" --mode "$mode" --steps 10 --warmup 3 --cpu-seconds 0 > "$O/ks_$mode.json" 2> "$O/ks_$mode.err" \
    || { echo "kernel trace $mode failed"; exit 1; }
  echo "kernel trace $mode ok"
done
for spec in "fwd tr_fwd" "mobilenet tr_mb"; do
  set -- $spec
  i=0
  for ctr in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$O/${2}_pmc_$i" -o pmc \
        -- python3 "$R/bench.py" --mode "$1" --steps 2 --warmup 1 --cpu-seconds 0 > "$O/${2}_pmc_$i.log" 2>&1 \
      || { echo "pmc $1 $ctr failed"; exit 1; }
    echo "pmc $1 $ctr ok"
  done
done
