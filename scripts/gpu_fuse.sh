#!/bin/bash
# MobileNet training fusions: parity, then AST bench fused vs unfused
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; OUT=$R/gpurun_out; mkdir -p $OUT
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mbtrain.py \
  tests/test_gpu_ast_train.py tests/test_gpu_determinism.py > $OUT/fuse_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $OUT/fuse_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 240 python3 bench.py --mode ast-train --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/fuse_bench.json 2> $OUT/fuse_bench.err || exit 1
AST_MBT_FUSE=0 timeout -k 10 240 python3 bench.py --mode ast-train --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/fuse_bench_off.json 2>> $OUT/fuse_bench.err || exit 1
for f in fuse_bench fuse_bench_off; do python3 -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',round(d['value'],1),round(d['ms_per_step'],2))"; done
