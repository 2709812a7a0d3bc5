#!/bin/bash
# Full GPU-box session: gpu_check.sh (tests, fwd bench, rocprof fwd) then the train and mobilenet
# benches and their rocprof kernel stats. Stops at the first failing step.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
TAG="${1:-full}"
bash "$ROOT/scripts/gpu_check.sh" "$TAG" || exit $?
cd "$ROOT"
for mode in train mobilenet ae-train; do
  timeout -k 10 600 python bench.py --mode $mode --steps 5 --warmup 2 --cpu-seconds 0 \
      > "$OUT/${TAG}_bench_$mode.json" 2> "$OUT/${TAG}_bench_$mode.err"
  rc=$?; echo "bench $mode rc=$rc"; cat "$OUT/${TAG}_bench_$mode.json"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
for mode in train mobilenet ae-train; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof_$mode" -o prof \
      -- python3 "$ROOT/bench.py" --mode $mode --steps 3 --warmup 1 --cpu-seconds 0 > "$OUT/${TAG}_prof_$mode.json" 2> "$OUT/${TAG}_prof_$mode.err"
  rc=$?; echo "rocprof $mode rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
