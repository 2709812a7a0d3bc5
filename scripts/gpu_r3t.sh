#!/bin/bash
# Hierarchical loss-accumulator arrival (det.h), reciprocal mvn passes, Gram kernels: full GPU
# suite, then config-3 / AST-train benches against libast_hip_gramprev.so (before these changes),
# alternating, and a kernel trace of config 3.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT/r3t
AST_TEST_DUMP=$OUT/r3t timeout -k 10 900 python3 -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -q -m gpu tests \
  > $OUT/r3t_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" $OUT/r3t_tests.log | tail -5; [ $rc -le 1 ] || exit $rc
P=$R/arbitrarystyletransfer_amd/libast_hip_gramprev.so
for rep in 1 2; do
  for m in train ast-train; do
    timeout -k 10 300 python3 bench.py --mode $m --cpu-seconds 0 > $OUT/r3t_${m}_new_$rep.json 2>> $OUT/r3t.err || exit 1
    AST_HIP_LIB=$P timeout -k 10 300 python3 bench.py --mode $m --cpu-seconds 0 > $OUT/r3t_${m}_prev_$rep.json 2>> $OUT/r3t.err || exit 1
    for v in new prev; do python3 -c "import json;d=json.load(open('$OUT/r3t_${m}_${v}_$rep.json'));print('$m $v rep $rep',round(d['value'],1),round(d['ms_per_step'],2))"; done
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/r3t_prof -o run -- python3 $R/bench.py --mode train --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/r3t_prof.log 2>&1 || exit 1
