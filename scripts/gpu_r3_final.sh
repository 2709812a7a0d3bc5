#!/bin/bash
# Round-3 closing session on the GPU box: full GPU suite, the bench lines of every mode (config 2 with
# its CPU baseline, as the driver runs it), then the rocprofv3 kernel-trace stats and the
# FETCH_SIZE / WRITE_SIZE passes behind the roofline fields (scripts/measure_profiles.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; R=$PWD; OUT=gpurun_out; mkdir -p $OUT; TAG="${1:-r03z}"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  # no -x: a failing test is recorded and the measurements still run (pytest exit 1 = failures;
  # anything else -- a timeout, an abort -- ends the session)
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
  rc=$?; grep -E "^FAILED|passed|failed" $OUT/${TAG}_tests.log | tail -5; [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 300 python bench.py > $OUT/${TAG}_bench_fwd.json 2> $OUT/${TAG}_bench_fwd.err || exit $?
cut -c1-300 $OUT/${TAG}_bench_fwd.json
for mode in mobilenet train ast-train ae-train; do
  timeout -k 10 300 python bench.py --mode $mode --cpu-seconds 0 > $OUT/${TAG}_bench_$mode.json 2> $OUT/${TAG}_bench_$mode.err || exit $?
  cut -c1-200 $OUT/${TAG}_bench_$mode.json
done
bash scripts/measure_profiles.sh ${TAG}m
