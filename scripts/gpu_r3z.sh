#!/bin/bash
# DP AutoEncoder step under concurrent GPU load (a config-3 bench in another process): does the
# result vary with scheduling? 6 runs, gradient hashes compared.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 200 python3 -u scripts/debug/dp_repeat.py 2 /tmp > $OUT/r3z_quiet.txt 2>&1 || exit 1
timeout -k 10 250 python3 bench.py --mode train --steps 400 --warmup 2 --cpu-seconds 0 > $OUT/r3z_load.json 2>&1 &
LP=$!
sleep 20
timeout -k 10 200 python3 -u scripts/debug/dp_repeat.py 6 /tmp > $OUT/r3z_loaded.txt 2>&1; rc=$?
kill $LP 2>/dev/null; wait $LP 2>/dev/null
grep -h "sha1\|worst" $OUT/r3z_quiet.txt $OUT/r3z_loaded.txt; exit $rc
