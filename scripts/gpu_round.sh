#!/bin/bash
# Round session on the GPU box: full GPU suite, bench lines (configs 2 and 5, CPU baselines), then the
# rocprofv3 kernel-trace stats and FETCH/WRITE_SIZE passes behind the roofline fields.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; R=$PWD; OUT=gpurun_out; mkdir -p $OUT; TAG="${1:-rnd}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
rc=$?; tail -3 $OUT/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/${TAG}_bench_fwd.json 2> $OUT/${TAG}_bench_fwd.err || exit $?
cat $OUT/${TAG}_bench_fwd.json
timeout -k 10 300 python bench.py --mode mobilenet > $OUT/${TAG}_bench_mobilenet.json 2> $OUT/${TAG}_bench_mobilenet.err || exit $?
cat $OUT/${TAG}_bench_mobilenet.json
timeout -k 10 200 python scripts/mb_launch_breakdown.py > $OUT/${TAG}_mb_launches.log 2>&1 || exit $?
bash scripts/measure_profiles.sh ${TAG}m
