#!/bin/bash
# Under concurrent GPU load: (1) the run-twice determinism tests; (2) the DP step with the wide GEMM
# off (AST_MBGEMM_WIDE=0), 6 runs.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 400 python3 bench.py --mode train --steps 900 --warmup 2 --cpu-seconds 0 > $OUT/r3z2_load.json 2>&1 &
LP=$!
sleep 20
timeout -k 10 200 python3 -u -m pytest -p no:cacheprovider --timeout 120 --timeout-method thread -q tests/test_gpu_determinism.py > $OUT/r3z2_det.log 2>&1
echo "det rc=$?"; grep -E "^FAILED|passed|failed" $OUT/r3z2_det.log | tail -8
AST_MBGEMM_WIDE=0 timeout -k 10 200 python3 -u scripts/debug/dp_repeat.py 6 /tmp > $OUT/r3z2_nowide.txt 2>&1; rc=$?
kill $LP 2>/dev/null; wait $LP 2>/dev/null
grep -h "sha1" $OUT/r3z2_nowide.txt; exit $rc
