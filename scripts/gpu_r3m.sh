#!/bin/bash
# Row-parallel mvn-Huber backward: training/loss parity + determinism, then config 3 (bench + kernel
# trace) and the trainers at the current tree.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -x -q \
  tests/test_gpu_training.py tests/test_gpu_determinism.py tests/test_gpu_parity.py tests/test_gpu_dispatch.py \
  tests/test_gpu_ast_train.py tests/test_gpu_mbtrain.py tests/test_gpu_hist.py > $OUT/r3m_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/r3m_tests.log; [ $rc -eq 0 ] || exit $rc
for m in train ast-train ae-train; do
  timeout -k 10 300 python3 bench.py --mode $m --cpu-seconds 0 > $OUT/r3m_$m.json 2>> $OUT/r3m.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/r3m_$m.json'));print('$m',round(d['value'],1),round(d['ms_per_step'],2))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r3m_ks_train" -o ks \
    -- python3 "$R/bench.py" --mode train --steps 5 --warmup 2 --cpu-seconds 0 > "$OUT/r3m_ks_train.json" 2> "$OUT/r3m_ks_train.err" \
  || { echo "kernel trace train failed"; exit 1; }
echo "kernel trace train ok"
