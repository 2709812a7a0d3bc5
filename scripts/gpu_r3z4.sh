#!/bin/bash
# Bisect the AdaIN forward variation under concurrent load (scripts/debug/race_probe2.py).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 300 python3 bench.py --mode train --steps 900 --warmup 2 --cpu-seconds 0 > $OUT/r3z4_load.json 2>&1 &
LP=$!
sleep 20
: > $OUT/r3z4.txt
timeout -k 10 100 python3 -u scripts/debug/race_probe2.py 12 >> $OUT/r3z4.txt 2>&1
AST_CONV_PACK=0 timeout -k 10 100 python3 -u scripts/debug/race_probe2.py 12 >> $OUT/r3z4.txt 2>&1
AST_CONV_M16=0 timeout -k 10 100 python3 -u scripts/debug/race_probe2.py 12 >> $OUT/r3z4.txt 2>&1
kill $LP 2>/dev/null; wait $LP 2>/dev/null
grep -v amdgpu.ids $OUT/r3z4.txt
