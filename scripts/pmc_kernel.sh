#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, no trace domains) over any python command:
#   bash scripts/pmc_kernel.sh <tag> <script.py> [args...]
# then: python scripts/pmc_kernel_summary.py <tag> <kernel-substring>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
TAG="$1"; shift
SCRIPT="$1"; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for group in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA" \
             "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $group --output-format csv -d "$OUT/${TAG}_pmc_$i" -o pmc \
      -- python3 "$ROOT/$SCRIPT" "$@" > "$OUT/${TAG}_pmc_$i.log" 2>&1
  rc=$?
  echo "pmc pass $i ($group) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/${TAG}_pmc_$i.log"; exit $rc; }
done
python3 "$ROOT/scripts/pmc_kernel_summary.py" "$TAG" "${PMC_KERNEL:-}" | tee "$OUT/${TAG}_pmc_summary.txt"
