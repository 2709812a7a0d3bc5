#!/bin/bash
# AdaAttN session: tests, the attention AST bench (config 5 geometry), rocprof kernel stats.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${1:-att}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_adaattn.py -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > "$OUT/${TAG}_tests.log" 2>&1
rc=$?; tail -2 "$OUT/${TAG}_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --mode mobilenet --attention --steps 5 --warmup 2 --cpu-seconds ${CPU_SECONDS:-15} \
    > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/${TAG}_bench.json"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof" -o prof \
    -- python3 "$ROOT/bench.py" --mode mobilenet --attention --steps 3 --warmup 1 --cpu-seconds 0 \
    > "$OUT/${TAG}_prof.json" 2> "$OUT/${TAG}_prof.err"
rc=$?; echo "rocprof rc=$rc"; exit $rc
