#!/bin/bash
# Kernel traces of the AST trainer step and config 5 at the current tree; config-3 bench (tv grid).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 300 python3 bench.py --mode train --cpu-seconds 0 > $OUT/r3x_train.json 2>> $OUT/r3x.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/r3x_train.json'));print('train',round(d['value'],1),round(d['ms_per_step'],2))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/r3x_prof_ast -o run -- python3 $R/bench.py --mode ast-train --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/r3x_prof_ast.log 2>&1 || exit 1
tail -1 $OUT/r3x_prof_ast.log | cut -c1-300
