#!/bin/bash
# dw kernels: parity tests, then the AST step breakdown
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mbtrain.py tests/test_gpu_determinism.py > $OUT/dw_tests.log 2>&1 || { tail -30 $OUT/dw_tests.log; exit 1; }
tail -3 $OUT/dw_tests.log
timeout -k 10 240 python3 scripts/debug/ast_gemm_shapes.py > $OUT/ast_shapes2.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_ast2 -o prof \
  -- python3 $R/bench.py --mode ast-train --steps 10 --warmup 2 --cpu-seconds 0 > $OUT/prof_ast2_bench.json 2> $OUT/prof_ast2.err
