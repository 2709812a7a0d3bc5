#!/bin/bash
# Round-3 GPU session: the determinism suite first (fails fast), then the whole GPU suite, then bench
# lines (configs 2, 3, 5 and the trainers) without the CPU baseline. Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; OUT=gpurun_out; mkdir -p $OUT; TAG="${1:-r3}"
PYT="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 $PYT tests/test_gpu_determinism.py -x -q > $OUT/${TAG}_det.log 2>&1
  rc=$?; tail -4 $OUT/${TAG}_det.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 900 $PYT tests -m gpu -q --deselect tests/test_gpu_determinism.py > $OUT/${TAG}_tests.log 2>&1
  rc=$?; tail -4 $OUT/${TAG}_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
for mode in ${MODES:-fwd mobilenet train ast-train ae-train}; do
  timeout -k 10 300 python bench.py --mode $mode --cpu-seconds 0 > $OUT/${TAG}_bench_$mode.json 2> $OUT/${TAG}_bench_$mode.err || exit $?
  cat $OUT/${TAG}_bench_$mode.json | cut -c1-400
done
