#!/bin/bash
# A/B of v4 expand+depthwise builds (AST_HIP_LIB=<variant .so>) over the config-5 launches
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; OUT=gpurun_out; mkdir -p $OUT; TAG="${1:-ab}"
for lib in arbitrarystyletransfer_amd/libast_hip.so ${LIBS:-}; do
  n=$(basename $lib .so)
  AST_HIP_LIB=$PWD/$lib timeout -k 10 200 python scripts/mb_launch_breakdown.py > $OUT/${TAG}_$n.log 2>&1 || exit $?
  echo "== $n"; grep -E "k5s1 40->240|k5s1 40->160 1024|k3s1 24->144 1024|k3s1 16->96 1024|k3s1 80->320 512|k5s1 96->384|256->768|128->384|pw 160->40 1024|pw 96->16|pw 240|pw 144|total_ms" $OUT/${TAG}_$n.log | sort -u -t, -k1,1 | cut -c1-80
done
