#!/bin/bash
# Kernel-trace stats of one bench mode under different environments, one rocprofv3 run per arm:
#   bash scripts/prof_ab.sh TAG MODE "name:VAR=val;VAR2=val" ["name2:..." ...]
# Writes gpurun_out/TAG_prof_<name>/ (rocprofv3 output) and prints per arm the 12 kernels with the
# largest total time (scripts/kernel_stats_top.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG="$1"; MODE="$2"; shift 2
for spec in "$@"; do
  name="${spec%%:*}"; envs="${spec#*:}"
  (
    IFS=';'; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof_$name -o run -- \
        python3 bench.py --mode "$MODE" --steps 10 --warmup 3 --cpu-seconds 0 > $OUT/${TAG}_prof_$name.json 2>&1
  ) || { echo "arm $name failed"; tail -5 $OUT/${TAG}_prof_$name.json; exit 1; }
  echo "== $name: $(tail -1 $OUT/${TAG}_prof_$name.json | cut -c1-160)"
  python3 scripts/kernel_stats_top.py $OUT/${TAG}_prof_$name 12
done
