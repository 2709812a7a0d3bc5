#!/bin/bash
# Which forward op varies under concurrent load (scripts/debug/race_probe.py).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 300 python3 bench.py --mode train --steps 900 --warmup 2 --cpu-seconds 0 > $OUT/r3z3_load.json 2>&1 &
LP=$!
sleep 20
timeout -k 10 200 python3 -u scripts/debug/race_probe.py 12 > $OUT/r3z3_probe.txt 2>&1; rc=$?
kill $LP 2>/dev/null; wait $LP 2>/dev/null
cat $OUT/r3z3_probe.txt | grep -v amdgpu.ids; exit $rc
