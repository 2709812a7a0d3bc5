#!/bin/bash
# PMC passes over one config-5 block (scripts/bench_mb_blocks.py <batch> <case-prefix>).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
CASE="${1:-dec8}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for group in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA" \
             "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_LEVEL_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d "$OUT/blk_${CASE}_pmc_$i" -o pmc \
      -- python3 "$ROOT/scripts/bench_mb_blocks.py" 32 "$CASE" > "$OUT/blk_${CASE}_pmc_$i.log" 2>&1
  rc=$?
  echo "pmc pass $i ($group) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/blk_${CASE}_pmc_$i.log"; exit $rc; }
done
