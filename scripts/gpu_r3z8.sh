#!/bin/bash
# cin4 plain stores + smallc lane shuffles: parity / determinism / training tests, the AdaIN forward
# stages and the 2-rank AE step beside a background bench, config-2 bench twice.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -q -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_determinism.py tests/test_gpu_training.py > $OUT/r3z8_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" $OUT/r3z8_tests.log | tail -5; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 bench.py --mode train --steps 1500 --warmup 2 --cpu-seconds 0 > $OUT/r3z8_load.json 2>&1 &
LP=$!
sleep 20
: > $OUT/r3z8.txt
timeout -k 10 100 python3 -u scripts/debug/race_probe2.py 16 >> $OUT/r3z8.txt 2>&1
timeout -k 10 250 python3 -u scripts/debug/dp_repeat.py 8 /tmp >> $OUT/r3z8.txt 2>&1
kill $LP 2>/dev/null; wait $LP 2>/dev/null
grep -v amdgpu.ids $OUT/r3z8.txt | grep -v "^   " | grep -v "keys differing from run 0: 0"
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --cpu-seconds 0 > $OUT/r3z8_fwd_$rep.json 2>> $OUT/r3z8.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/r3z8_fwd_$rep.json'));print('fwd rep $rep',round(d['value'],1),round(d['ms_per_step'],3))"
done
