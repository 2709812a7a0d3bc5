#!/bin/bash
# MobileNet parity tests on the default build, then the A/B launch breakdown over variant builds
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; OUT=gpurun_out; mkdir -p $OUT; TAG="${1:-mbab}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_mobilenet.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_tests.log 2>&1
rc=$?; tail -3 $OUT/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ed4_ab.sh $TAG
