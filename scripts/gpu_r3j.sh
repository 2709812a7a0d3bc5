#!/bin/bash
# VALU-rate microbenchmark, k5 dot2 variant (parity + A/B), k5 3-wave variant A/B, AST conv tuning.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd $R
bash scripts/gpu_r3i.sh || exit $?
bash scripts/gpu_r3h.sh || exit $?
