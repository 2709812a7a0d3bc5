#!/bin/bash
# Effective clock and MFMA-pipe busy fraction of the conv3x3 dispatches of a bench mode (DVFS
# give-back, MI355X_MICROARCH.md): one rocprofv3 pass with GRBM_GUI_ACTIVE, SQ_VALU_MFMA_BUSY_CYCLES,
# SQ_BUSY_CYCLES and the kernel trace (durations), then scripts/pmc_clock_summary.py.
#   bash scripts/pmc_clock.sh TAG [mode] [kernel-substring]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; MODE="${2:-fwd}"; KS="${3:-conv3x3}"
O="$ROOT/gpurun_out/${TAG}_clock"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace \
    --output-format csv -d "$O" -o clk -- python3 "$ROOT/bench.py" --mode "$MODE" --steps 4 --warmup 2 \
    --cpu-seconds 0 > "$O/run.log" 2>&1 || { echo "pmc clock pass failed"; tail -5 "$O/run.log"; exit 1; }
python3 "$ROOT/scripts/pmc_clock_summary.py" "$O" "$KS"
