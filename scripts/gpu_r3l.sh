#!/bin/bash
# Row-parallel elementwise backward kernels + split-bf16 triangle Gram: parity, then the config-3
# bench with AST_BWD_ROWPAR=1/0 and AST_GRAM_X3=1/0 (alternating), the AST / AE trainers.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -x -q \
  tests/test_gpu_training.py tests/test_gpu_determinism.py tests/test_gpu_parity.py tests/test_gpu_dispatch.py \
  tests/test_gpu_ast_train.py tests/test_gpu_mbtrain.py > $OUT/r3l_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/r3l_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in "1 1" "0 1" "1 0" "0 0"; do
  set -- $cfg
  AST_BWD_ROWPAR=$1 AST_GRAM_X3=$2 timeout -k 10 300 python3 bench.py --mode train --cpu-seconds 0 > $OUT/r3l_train_$1$2.json 2>> $OUT/r3l.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/r3l_train_$1$2.json'));print('train rowpar=$1 gram_x3=$2',round(d['value'],1),round(d['ms_per_step'],2))"
done
for m in ast-train ae-train; do
  timeout -k 10 300 python3 bench.py --mode $m --cpu-seconds 0 > $OUT/r3l_$m.json 2>> $OUT/r3l.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/r3l_$m.json'));print('$m',round(d['value'],1),round(d['ms_per_step'],2))"
done
