"""Summarise scripts/pmc_block.sh output: mean per-dispatch counters per kernel family."""
import collections
import csv
import glob
import sys

case = sys.argv[1] if len(sys.argv) > 1 else "dec8"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(collections.Counter)
for f in sorted(glob.glob(f"gpurun_out/blk_{case}_pmc_*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        kk = "expand_dw" if "expand_dw" in k else "pw" if "pw_kernel" in k else None
        if kk:
            agg[kk][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[kk][r["Counter_Name"]] += 1
for kk, d in agg.items():
    m = {c: v / cnt[kk][c] for c, v in d.items()}
    w = m.get("SQ_WAVES", 1)
    print(f"{kk}: waves {w:.0f}  VALU/wave {m.get('SQ_INSTS_VALU', 0) / w:.0f}  SALU/wave {m.get('SQ_INSTS_SALU', 0) / w:.0f}"
          f"  LDS/wave {m.get('SQ_INSTS_LDS', 0) / w:.0f}  MFMA/wave {m.get('SQ_INSTS_MFMA', 0) / w:.0f}"
          f"  VMEM rd/wr per wave {m.get('SQ_INSTS_VMEM_RD', 0) / w:.0f}/{m.get('SQ_INSTS_VMEM_WR', 0) / w:.0f}")
    wc = m.get("SQ_WAVE_CYCLES", 1)
    print(f"   wave-cycles: busy-inst-any {m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f}  valu {m.get('SQ_ACTIVE_INST_VALU', 0) / wc:.2f}"
          f"  lds {m.get('SQ_ACTIVE_INST_LDS', 0) / wc:.2f}  wait-any {m.get('SQ_WAIT_ANY', 0) / wc:.2f}"
          f"  wait-inst-any {m.get('SQ_WAIT_INST_ANY', 0) / wc:.2f}  wait-lds {m.get('SQ_WAIT_INST_LDS', 0) / wc:.2f}")
    print(f"   LDS bank conflict / LDS active {m.get('SQ_LDS_BANK_CONFLICT', 0) / max(m.get('SQ_LDS_IDX_ACTIVE', 1), 1):.2f}"
          f"  GRBM_GUI_ACTIVE {m.get('GRBM_GUI_ACTIVE', 0):.3g}  wave-cycles/wave {wc / w:.0f}")
