#!/bin/bash
# The DP AutoEncoder golden test inside the mbtrain test file (where it failed twice), with the
# ranks' results kept (AST_TEST_DUMP), and one standalone run for reference.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT/r3v
timeout -k 10 200 python3 -u scripts/debug/dp_repeat.py 1 $OUT/r3v > $OUT/r3v_standalone.txt 2>&1 || exit 1
AST_TEST_DUMP=$OUT/r3v timeout -k 10 600 python3 -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -q \
  tests/test_gpu_mbtrain.py tests/test_gpu_ast_train.py > $OUT/r3v_tests.log 2>&1
echo "tests rc=$?"; tail -3 $OUT/r3v_tests.log; cat $OUT/r3v_standalone.txt
