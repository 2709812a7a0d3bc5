#!/bin/bash
# Wide-N training GEMM: parity (mbtrain, AE / AST steps, determinism), the shape probe, AST / AE
# benches with AST_MBGEMM_WIDE=1 / 0.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -x -q \
  tests/test_gpu_mbtrain.py tests/test_gpu_ast_train.py tests/test_gpu_determinism.py > $OUT/r3o_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/r3o_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/debug/gemm_probe.py > $OUT/r3o_gemm_probe.txt 2>&1 || exit 1
cat $OUT/r3o_gemm_probe.txt
for w in 1 0; do
  for m in ast-train ae-train; do
    AST_MBGEMM_WIDE=$w timeout -k 10 300 python3 bench.py --mode $m --cpu-seconds 0 > $OUT/r3o_${m}_w$w.json 2>> $OUT/r3o.err || exit 1
    python3 -c "import json;d=json.load(open('$OUT/r3o_${m}_w$w.json'));print('$m wide=$w',round(d['value'],1),round(d['ms_per_step'],2),d['mbgemm_tflops'])"
  done
done
