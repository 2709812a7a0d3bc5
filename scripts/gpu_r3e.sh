#!/bin/bash
# 512^2 training-step gradients vs a float64 oracle; config-3 kernel trace; AST GEMM shapes.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -q -s --timeout 380 --timeout-method thread \
  tests/test_gpu_training.py -k "512" > $OUT/r3e_512.log 2>&1
rc=$?; echo "512 test rc=$rc"; grep -E "grad |512\^2|passed|failed|Error" $OUT/r3e_512.log | tail -40
[ $rc -le 1 ] || exit $rc
timeout -k 10 240 python3 scripts/debug/ast_gemm_shapes.py > $OUT/r3e_ast_shapes.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r3e_ks_train" -o ks \
    -- python3 "$R/bench.py" --mode train --steps 5 --warmup 2 --cpu-seconds 0 > "$OUT/r3e_ks_train.json" 2> "$OUT/r3e_ks_train.err" \
  || { echo "kernel trace train failed"; exit 1; }
echo "kernel trace train ok"
