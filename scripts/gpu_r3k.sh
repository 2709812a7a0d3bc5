#!/bin/bash
# Split-bf16 triangle Gram: parity (gram, losses, determinism, torch.ops), then config-3 / AST / AE
# benches with AST_GRAM_X3=1 (default) and 0.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -x -q \
  tests/test_gpu_training.py tests/test_gpu_determinism.py tests/test_gpu_parity.py tests/test_gpu_dispatch.py \
  tests/test_gpu_ast_train.py tests/test_gpu_mbtrain.py > $OUT/r3k_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/r3k_tests.log; [ $rc -eq 0 ] || exit $rc
for x in 1 0; do
  AST_GRAM_X3=$x timeout -k 10 300 python3 bench.py --mode train --cpu-seconds 0 > $OUT/r3k_train_x$x.json 2>> $OUT/r3k.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/r3k_train_x$x.json'));print('train gram_x3=$x',round(d['value'],1),round(d['ms_per_step'],2))"
done
for m in ast-train ae-train; do
  timeout -k 10 300 python3 bench.py --mode $m --cpu-seconds 0 > $OUT/r3k_$m.json 2>> $OUT/r3k.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/r3k_$m.json'));print('$m',round(d['value'],1),round(d['ms_per_step'],2))"
done
