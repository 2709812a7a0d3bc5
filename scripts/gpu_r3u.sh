#!/bin/bash
# DP AutoEncoder step after the GPU has been loaded (hot clocks): bit-identical across runs?
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 300 python3 bench.py --mode train --steps 60 --cpu-seconds 0 > $OUT/r3u_warm.json 2>> $OUT/r3u.err || exit 1
timeout -k 10 400 python3 -u scripts/debug/dp_repeat.py 4 /tmp > $OUT/r3u_dp.txt 2>&1; rc=$?
cat $OUT/r3u_dp.txt; exit $rc
