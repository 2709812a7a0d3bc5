#!/bin/bash
# AE data-parallel golden step with the wide GEMM off / on
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
for w in 0 1; do
  AST_MBGEMM_WIDE=$w timeout -k 10 300 python3 -u -m pytest -p no:cacheprovider --timeout 240 --timeout-method thread -x -q \
    tests/test_gpu_mbtrain.py -k "dp_syncbn or autoencoder_step" > $OUT/r3p_w$w.log 2>&1
  echo "wide=$w rc=$?"; grep -E "passed|failed|^E  " $OUT/r3p_w$w.log | head -5
done
