#!/bin/bash
# A/B of the split-bf16 conv on the 32x32x16 (AST_CONV_M16=0) vs 16x16x32 (=1) MFMA, alternating runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; OUT=gpurun_out; mkdir -p $OUT
for r in 1 2; do
  for m in 0 1; do
    AST_CONV_M16=$m timeout -k 10 120 python bench.py --cpu-seconds 0 ${ARGS:-} > $OUT/ab_m16_${m}_$r.json 2>/dev/null || exit $?
    python -c "import json,sys; d=json.load(open('$OUT/ab_m16_${m}_$r.json')); print('M16=$m run $r', round(d['value'],1), 'img/s', round(d['roofline']['achieved'],1), 'TF', round(d['roofline']['frac'],3))"
  done
done
