#!/bin/bash
# After removing the cin4 nontemporal stores: encoder layer walk (16 repeats), AdaIN forward
# stages, and the 2-rank AE step (8 runs), all beside a background config-3 bench.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 400 python3 bench.py --mode train --steps 1500 --warmup 2 --cpu-seconds 0 > $OUT/r3z6_load.json 2>&1 &
LP=$!
sleep 20
: > $OUT/r3z6.txt
timeout -k 10 100 python3 -u scripts/debug/race_probe3.py 16 >> $OUT/r3z6.txt 2>&1
timeout -k 10 100 python3 -u scripts/debug/race_probe2.py 16 >> $OUT/r3z6.txt 2>&1
timeout -k 10 250 python3 -u scripts/debug/dp_repeat.py 8 /tmp >> $OUT/r3z6.txt 2>&1; rc=$?
kill $LP 2>/dev/null; wait $LP 2>/dev/null
grep -v amdgpu.ids $OUT/r3z6.txt | grep -v "^   "; exit $rc
