#!/bin/bash
# Split-plane content / style-moment losses: parity (training losses, AE / AST steps, determinism),
# then config-3 (--mode train) and AST-train benches with AST_PLANE_SPLIT=1 / 0, alternating.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -x -q \
  tests/test_gpu_training.py tests/test_gpu_determinism.py tests/test_gpu_ast_train.py > $OUT/r3r_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/r3r_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    for m in train ast-train; do
      AST_PLANE_SPLIT=$v timeout -k 10 300 python3 bench.py --mode $m --cpu-seconds 0 > $OUT/r3r_${m}_s${v}_$rep.json 2>> $OUT/r3r.err || exit 1
      python3 -c "import json;d=json.load(open('$OUT/r3r_${m}_s${v}_$rep.json'));print('$m split=$v rep $rep',round(d['value'],1),round(d['ms_per_step'],2))"
    done
  done
done
