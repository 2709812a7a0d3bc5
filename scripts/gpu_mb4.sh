#!/bin/bash
# v4 expand+depthwise session: MobileNet parity tests, per-launch breakdown, config-5 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; OUT=gpurun_out; mkdir -p $OUT; TAG="${1:-mb4}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_mobilenet.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_tests.log 2>&1
rc=$?; tail -3 $OUT/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/mb_launch_breakdown.py > $OUT/${TAG}_launches.log 2>&1 || exit $?
grep -v amdgpu $OUT/${TAG}_launches.log | head -30
timeout -k 10 300 python bench.py --mode mobilenet --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err
rc=$?; cat $OUT/${TAG}_bench.json; exit $rc
