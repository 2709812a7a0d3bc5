#!/bin/bash
# Layer-by-layer encoder probe under concurrent load (scripts/debug/race_probe3.py), default and
# AST_CONV_PACK=0.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 300 python3 bench.py --mode train --steps 900 --warmup 2 --cpu-seconds 0 > $OUT/r3z5_load.json 2>&1 &
LP=$!
sleep 20
: > $OUT/r3z5.txt
timeout -k 10 100 python3 -u scripts/debug/race_probe3.py 16 >> $OUT/r3z5.txt 2>&1
echo "-- AST_CONV_PACK=0" >> $OUT/r3z5.txt
AST_CONV_PACK=0 timeout -k 10 100 python3 -u scripts/debug/race_probe3.py 16 >> $OUT/r3z5.txt 2>&1
kill $LP 2>/dev/null; wait $LP 2>/dev/null
grep -v amdgpu.ids $OUT/r3z5.txt
