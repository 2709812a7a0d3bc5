#!/bin/bash
# Round-3 survey: M16 conv A/B on config 2, split-bf16 1x1 GEMM A/B on the AST trainer, kernel-trace
# stats of the fwd / mobilenet / ast-train / ae-train benches.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R; OUT=$R/gpurun_out; mkdir -p $OUT
bash scripts/gpu_ab_m16.sh || exit $?
for x in 0 1; do
  AST_MBGEMM_X3=$x timeout -k 10 240 python3 bench.py --mode ast-train --cpu-seconds 0 > $OUT/r3d_ast_x3_$x.json 2>> $OUT/r3d.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/r3d_ast_x3_$x.json'));print('ast x3=$x',round(d['value'],1),round(d['ms_per_step'],2),d['mbgemm_tflops'])"
done
timeout -k 10 240 python3 bench.py --mode ae-train --cpu-seconds 0 > $OUT/r3d_ae.json 2>> $OUT/r3d.err || exit 1
cd /tmp && export TMPDIR=/tmp
for mode in fwd mobilenet ast-train ae-train; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r3d_ks_$mode" -o ks \
      -- python3 "$R/bench.py" --mode "$mode" --steps 10 --warmup 3 --cpu-seconds 0 > "$OUT/r3d_ks_$mode.json" 2> "$OUT/r3d_ks_$mode.err" \
    || { echo "kernel trace $mode failed"; exit 1; }
  echo "kernel trace $mode ok"
done
