#!/bin/bash
# Pairwise content+style loss op, capped loss-kernel grids: training / AST / AE / hist / dispatcher
# tests, then config-3 and AST-train benches and a config-3 kernel trace; the DP step probe (CUs).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT/r3w
timeout -k 10 200 python3 -u scripts/debug/dp_repeat.py 1 $OUT/r3w > $OUT/r3w_dp.txt 2>&1 || exit 1
cat $OUT/r3w_dp.txt; rm -f $OUT/r3w/dp_0.npz
AST_TEST_DUMP=$OUT/r3w timeout -k 10 900 python3 -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -q -m gpu tests \
  > $OUT/r3w_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" $OUT/r3w_tests.log | tail -5; [ $rc -le 1 ] || exit $rc
for rep in 1 2; do
  for m in train ast-train; do
    timeout -k 10 300 python3 bench.py --mode $m --cpu-seconds 0 > $OUT/r3w_${m}_$rep.json 2>> $OUT/r3w.err || exit 1
    python3 -c "import json;d=json.load(open('$OUT/r3w_${m}_$rep.json'));print('$m rep $rep',round(d['value'],1),round(d['ms_per_step'],2))"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/r3w_prof -o run -- python3 $R/bench.py --mode train --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/r3w_prof.log 2>&1 || exit 1
