#!/bin/bash
# k5 depthwise taps on bf16 v_dot2 (libast_hip_dot2.so, ED4_DOT2=1) vs the default fp32-FMA build:
# the config-5 bf16 parity tests on the variant, then the config-5 bench alternating.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
V=$R/arbitrarystyletransfer_amd/libast_hip_dot2.so
AST_HIP_LIB=$V timeout -k 10 400 python3 -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -x -q \
  tests/test_gpu_mobilenet.py -k "bf16 or golden or config5" > $OUT/r3i_tests.log 2>&1
rc=$?; echo "dot2 tests rc=$rc"; tail -3 $OUT/r3i_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 240 python3 bench.py --mode mobilenet --cpu-seconds 0 > $OUT/r3i_mb_def$r.json 2>> $OUT/r3i.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/r3i_mb_def$r.json'));print('default',round(d['value'],1),round(d['ms_per_step'],2))"
  AST_HIP_LIB=$V timeout -k 10 240 python3 bench.py --mode mobilenet --cpu-seconds 0 > $OUT/r3i_mb_dot2$r.json 2>> $OUT/r3i.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/r3i_mb_dot2$r.json'));print('k5 dot2',round(d['value'],1),round(d['ms_per_step'],2))"
done
