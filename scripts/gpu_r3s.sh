#!/bin/bash
# Gram forward (diagonal tiles read once, idle lower quadrant, register prefetch) and Gram backward
# (register prefetch): parity, then config-3 benches against the previous kernels' build
# (libast_hip_gramprev.so via AST_HIP_LIB), alternating.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -x -q \
  tests/test_gpu_training.py tests/test_gpu_determinism.py tests/test_gpu_ast_train.py > $OUT/r3s_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/r3s_tests.log; [ $rc -eq 0 ] || exit $rc
P=$R/arbitrarystyletransfer_amd/libast_hip_gramprev.so
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --mode train --cpu-seconds 0 > $OUT/r3s_train_new_$rep.json 2>> $OUT/r3s.err || exit 1
  AST_HIP_LIB=$P timeout -k 10 300 python3 bench.py --mode train --cpu-seconds 0 > $OUT/r3s_train_prev_$rep.json 2>> $OUT/r3s.err || exit 1
  for v in new prev; do python3 -c "import json;d=json.load(open('$OUT/r3s_train_${v}_$rep.json'));print('train $v rep $rep',round(d['value'],1),round(d['ms_per_step'],2))"; done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/r3s_prof -o run -- python3 $R/bench.py --mode train --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/r3s_prof.log 2>&1 || exit 1
find $OUT/r3s_prof -name "*kernel_stats.csv" -exec cp {} $OUT/r3s_kernel_stats_train.csv \;
