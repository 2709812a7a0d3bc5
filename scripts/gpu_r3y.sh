#!/bin/bash
# AST trainer: stylized and org_out through the loss network in one pass; parity and bench.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -q \
  tests/test_gpu_ast_train.py tests/test_gpu_determinism.py > $OUT/r3y_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" $OUT/r3y_tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --mode ast-train --cpu-seconds 0 > $OUT/r3y_ast_$rep.json 2>> $OUT/r3y.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/r3y_ast_$rep.json'));print('ast-train rep $rep',round(d['value'],1),round(d['ms_per_step'],2))"
done
