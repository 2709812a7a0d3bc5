#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel stats. Stops at the first step that
# crashes or times out (exit codes other than 0/1 from pytest, anything non-zero afterwards).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
TAG="${1:-run}"
STEPS="${BENCH_STEPS:-10}"

timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1
rc=$?
echo "gpu tests rc=$rc"; tail -5 "$OUT/${TAG}_tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi

BENCH_PER_LAYER=1 timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 3 --cpu-seconds "${CPU_SECONDS:-10}" \
    > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
rc=$?
echo "bench rc=$rc"; cat "$OUT/${TAG}_bench.json"; tail -3 "$OUT/${TAG}_bench.err"
[ $rc -eq 0 ] || exit $rc

if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof" -o prof \
      -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --cpu-seconds 0 > "$OUT/${TAG}_prof_bench.json" 2> "$OUT/${TAG}_prof.err"
  rc=$?
  echo "rocprof rc=$rc"
  find "$OUT/${TAG}_prof" -name "*stats*" | head
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
