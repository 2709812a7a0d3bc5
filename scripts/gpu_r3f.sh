#!/bin/bash
# Fused MobileNet block pair: parity + config-5 A/B; 512^2 gradients vs float64; config-3 trace;
# AST GEMM shapes.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
PYT="python3 -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 400 $PYT -x -q tests/test_gpu_mobilenet.py tests/test_gpu_determinism.py > $OUT/r3f_mb.log 2>&1
rc=$?; echo "mobilenet tests rc=$rc"; tail -4 $OUT/r3f_mb.log; [ $rc -eq 0 ] || exit $rc
for e in 1 0; do
  AST_MB_EDPW=$e timeout -k 10 240 python3 bench.py --mode mobilenet --cpu-seconds 0 > $OUT/r3f_mb_edpw$e.json 2>> $OUT/r3f.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/r3f_mb_edpw$e.json'));print('edpw=$e',round(d['value'],1),round(d['ms_per_step'],2),round(d['roofline']['whole_step']['frac'],4))"
done
timeout -k 10 500 $PYT -x -q -s tests/test_gpu_training.py -k "512" > $OUT/r3f_512.log 2>&1
rc=$?; echo "512 test rc=$rc"; grep -E "grad |512\^2|passed|failed|Error" $OUT/r3f_512.log | tail -40
[ $rc -le 1 ] || exit $rc
timeout -k 10 240 python3 scripts/debug/ast_gemm_shapes.py > $OUT/r3f_ast_shapes.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r3f_ks_train" -o ks \
    -- python3 "$R/bench.py" --mode train --steps 5 --warmup 2 --cpu-seconds 0 > "$OUT/r3f_ks_train.json" 2> "$OUT/r3f_ks_train.err" \
  || { echo "kernel trace train failed"; exit 1; }
echo "kernel trace train ok"
