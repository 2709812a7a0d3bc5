#!/bin/bash
# MobileNet kernel session: bf16/fp32 block parity tests, then per-block timing for the v1 and v2
# expand+depthwise kernels (AST_MB_ED=1/2), then the config-5 bench.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; TAG="${1:-mb}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_mobilenet.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/${TAG}_tests.log" 2>&1
rc=$?; tail -3 "$OUT/${TAG}_tests.log"; [ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-"AST_MB_ED=1" "AST_MB_ED=2"}; do
  env $v timeout -k 10 300 python scripts/bench_mb_blocks.py 32 > "$OUT/${TAG}_blocks_$v.log" 2>&1
  rc=$?; echo "$v"; grep -v amdgpu.ids "$OUT/${TAG}_blocks_$v.log"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python bench.py --mode mobilenet --steps 5 --warmup 2 --cpu-seconds 0 > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
rc=$?; cat "$OUT/${TAG}_bench.json"; exit $rc
