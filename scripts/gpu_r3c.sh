#!/bin/bash
# training-path parity (AdaIN / AE / AST), then the AST step breakdown and benches (x3 / fp32 GEMM)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_training.py \
  tests/test_gpu_mbtrain.py tests/test_gpu_ast_train.py tests/test_gpu_dispatch.py > $OUT/r3c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $OUT/r3c_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 240 python3 scripts/debug/ast_gemm_shapes.py > $OUT/ast_shapes3.txt 2>&1 || exit 1
timeout -k 10 240 python3 bench.py --mode ast-train --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/x3g_bench.json 2> $OUT/x3g_bench.err || exit 1
AST_MBGEMM_X3=0 timeout -k 10 240 python3 bench.py --mode ast-train --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/x3g_bench_fp32.json 2>> $OUT/x3g_bench.err
