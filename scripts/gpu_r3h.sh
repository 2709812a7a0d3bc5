#!/bin/bash
# k5 expand+depthwise at 3 waves/SIMD (spilling build, libast_hip_w3.so) vs the default build, config 5.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 60 ./scripts/microbench/valu_rate > $OUT/r3h_valu_rate.txt 2>&1 || exit 1
cat $OUT/r3h_valu_rate.txt
for r in 1 2; do
  timeout -k 10 240 python3 bench.py --mode mobilenet --cpu-seconds 0 > $OUT/r3h_mb_def$r.json 2>> $OUT/r3h.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/r3h_mb_def$r.json'));print('default',round(d['value'],1),round(d['ms_per_step'],2))"
  AST_HIP_LIB=$R/arbitrarystyletransfer_amd/libast_hip_w3.so timeout -k 10 240 python3 bench.py --mode mobilenet --cpu-seconds 0 > $OUT/r3h_mb_w3$r.json 2>> $OUT/r3h.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/r3h_mb_w3$r.json'));print('k5 w3',round(d['value'],1),round(d['ms_per_step'],2))"
done
# conv3x3 configurations for the ASTTrainer step's shapes (loss network on packed small planes)
timeout -k 10 400 env TUNE_AST=1 TUNE_NEW=1 TUNE_COPY=$OUT/conv_tuning_ast.json python3 scripts/tune_conv.py > $OUT/r3h_tune_ast.log 2>&1 || exit 1
tail -1 $OUT/r3h_tune_ast.log
timeout -k 10 240 python3 bench.py --mode ast-train --cpu-seconds 0 > $OUT/r3h_ast_tuned.json 2>> $OUT/r3h.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/r3h_ast_tuned.json'));print('ast tuned',round(d['value'],1),round(d['ms_per_step'],2))"
