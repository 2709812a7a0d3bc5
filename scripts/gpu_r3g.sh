#!/bin/bash
# Fused MobileNet pair (occupancy fix) A/B + parity; streaming 1x1 training GEMM parity + AST/AE benches.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
PYT="python3 -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 400 $PYT -x -q tests/test_gpu_mobilenet.py -k "fused or block_bf16" tests/test_gpu_mbtrain.py > $OUT/r3g_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $OUT/r3g_tests.log; [ $rc -eq 0 ] || exit $rc
for e in 1 0; do
  AST_MB_EDPW=$e timeout -k 10 240 python3 bench.py --mode mobilenet --cpu-seconds 0 > $OUT/r3g_mb_edpw$e.json 2>> $OUT/r3g.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/r3g_mb_edpw$e.json'));print('edpw=$e',round(d['value'],1),round(d['ms_per_step'],2),round(d['roofline']['whole_step']['frac'],4))"
done
for e in 1 0; do
  AST_MBGEMM_PW1=$e timeout -k 10 240 python3 bench.py --mode ast-train --cpu-seconds 0 > $OUT/r3g_ast_pw1$e.json 2>> $OUT/r3g.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/r3g_ast_pw1$e.json'));print('ast pw1=$e',round(d['value'],1),round(d['ms_per_step'],2),d['mbgemm_tflops'])"
  AST_MBGEMM_PW1=$e timeout -k 10 240 python3 bench.py --mode ae-train --cpu-seconds 0 > $OUT/r3g_ae_pw1$e.json 2>> $OUT/r3g.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/r3g_ae_pw1$e.json'));print('ae pw1=$e',round(d['value'],1),round(d['ms_per_step'],2),d['mbgemm_tflops'])"
done
