#!/bin/bash
# Aligned-load pad_grad / pad-upsample adjoint: training parity + determinism, config-3 bench and trace;
# the 1x1 training GEMM shape probe.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -x -q \
  tests/test_gpu_training.py tests/test_gpu_determinism.py tests/test_gpu_ast_train.py tests/test_gpu_mbtrain.py \
  > $OUT/r3n_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/r3n_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --mode train --cpu-seconds 0 > $OUT/r3n_train.json 2>> $OUT/r3n.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/r3n_train.json'));print('train',round(d['value'],1),round(d['ms_per_step'],2))"
timeout -k 10 200 python3 scripts/debug/gemm_probe.py > $OUT/r3n_gemm_probe.txt 2>&1 || exit 1
cat $OUT/r3n_gemm_probe.txt
AST_MBGEMM_X3=1 timeout -k 10 200 python3 scripts/debug/gemm_probe.py > $OUT/r3n_gemm_probe_x3.txt 2>&1 || exit 1
cat $OUT/r3n_gemm_probe_x3.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r3n_ks_train" -o ks \
    -- python3 "$R/bench.py" --mode train --steps 5 --warmup 2 --cpu-seconds 0 > "$OUT/r3n_ks_train.json" 2> "$OUT/r3n_ks_train.err" \
  || { echo "kernel trace train failed"; exit 1; }
echo "kernel trace train ok"
