#!/bin/bash
# rocprofv3 hardware-counter passes over a short bench run (one counter group per pass; no trace
# domains combined with --pmc). Output under gpurun_out/<tag>_pmc_*; summary via pmc_summary.py.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
TAG="${1:-pmc}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/${TAG}_counters_list.txt" 2>&1 || echo "counter list failed (ignored)"
i=0
for group in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d "$OUT/${TAG}_pmc_$i" -o pmc \
      -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-seconds 0 > "$OUT/${TAG}_pmc_$i.log" 2>&1
  rc=$?
  echo "pmc pass $i ($group) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/${TAG}_pmc_$i.log"; exit $rc; }
done
python3 "$ROOT/scripts/pmc_summary.py" "$OUT" "$TAG" | tee "$OUT/${TAG}_summary.json"
