#!/bin/bash
# M16 conv A/B (bench, alternating) + the AST-trainer graph test + ast-train bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; OUT=gpurun_out; mkdir -p $OUT
bash scripts/gpu_ab_m16.sh || exit $?
timeout -k 10 300 python -u -m pytest -p no:cacheprovider -q -x --timeout 240 --timeout-method thread \
  tests/test_gpu_ast_train.py tests/test_gpu_parity.py -k "graph or nonfinite or torch_ops" > $OUT/r3b_tests.log 2>&1
rc=$?; tail -5 $OUT/r3b_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --mode ast-train --cpu-seconds 0 > $OUT/r3b_bench_ast.json 2> $OUT/r3b_bench_ast.err || exit $?
cut -c1-600 $OUT/r3b_bench_ast.json
