#!/bin/bash
# rocprofv3 kernel-trace stats of the ASTTrainer step (graph mode) and the AE step
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_ast -o prof \
  -- python3 $R/bench.py --mode ast-train --steps 10 --warmup 2 --cpu-seconds 0 > $OUT/prof_ast_bench.json 2> $OUT/prof_ast.err || exit $?
find $OUT/prof_ast -name "*kernel_stats.csv" | head -3
