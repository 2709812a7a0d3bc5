#!/bin/bash
# After the cin4 nontemporal-store removal: conv / style-transfer parity tests, determinism, config 2
# bench (conv_1 ran nontemporal stores there) twice.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -q -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_determinism.py tests/test_gpu_training.py > $OUT/r3z7_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" $OUT/r3z7_tests.log | tail -5; [ $rc -le 1 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --cpu-seconds 0 > $OUT/r3z7_fwd_$rep.json 2>> $OUT/r3z7.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/r3z7_fwd_$rep.json'));print('fwd rep $rep',round(d['value'],1),round(d['ms_per_step'],3))"
done
