"""Summarise scripts/pmc_kernel.sh output: mean per-dispatch counters per kernel (name filter)."""
import collections
import csv
import glob
import os
import sys

tag = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(collections.Counter)
for f in sorted(glob.glob(os.path.join(root, f"{tag}_pmc_*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if filt and filt not in k:
            continue
        k = k.replace("(anonymous namespace)::", "").removeprefix("void ").split("(")[0][-60:]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
for kk, d in agg.items():
    m = {c: v / cnt[kk][c] for c, v in d.items()}
    w = max(m.get("SQ_WAVES", 1), 1)
    wc = max(m.get("SQ_WAVE_CYCLES", 1), 1)
    print(f"{kk}: dispatches {max(cnt[kk].values())}  waves {w:.0f}")
    print(f"   per wave: VALU {m.get('SQ_INSTS_VALU', 0) / w:.0f}  SALU {m.get('SQ_INSTS_SALU', 0) / w:.0f}  LDS "
          f"{m.get('SQ_INSTS_LDS', 0) / w:.0f}  MFMA {m.get('SQ_INSTS_MFMA', 0) / w:.0f}  VMEM rd/wr "
          f"{m.get('SQ_INSTS_VMEM_RD', 0) / w:.0f}/{m.get('SQ_INSTS_VMEM_WR', 0) / w:.0f}  wave-cycles {wc / w:.0f}")
    print(f"   fraction of wave-cycles: inst-any {m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f}  valu "
          f"{m.get('SQ_ACTIVE_INST_VALU', 0) / wc:.2f}  lds {m.get('SQ_ACTIVE_INST_LDS', 0) / wc:.2f}  misc "
          f"{m.get('SQ_ACTIVE_INST_MISC', 0) / wc:.2f}  wait-any {m.get('SQ_WAIT_ANY', 0) / wc:.2f}  wait-inst-any "
          f"{m.get('SQ_WAIT_INST_ANY', 0) / wc:.2f}  wait-lds {m.get('SQ_WAIT_INST_LDS', 0) / wc:.2f}")
    print(f"   LDS bank-conflict cycles / LDS active {m.get('SQ_LDS_BANK_CONFLICT', 0) / max(m.get('SQ_LDS_IDX_ACTIVE', 1), 1):.3f}"
          # SQ_VALU_MFMA_BUSY_CYCLES sums every SIMD's MFMA cycles; GRBM_GUI_ACTIVE sums the 8 XCDs'
          # clocks (MI355X_MICROARCH.md): busy fraction = busy / (GRBM / 8 * 1024 SIMDs)
          f"  MFMA busy per SIMD-cycle {m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / max(m.get('GRBM_GUI_ACTIVE', 1) / 8 * 1024, 1):.3f}"
          f"  FETCH_SIZE {m.get('FETCH_SIZE', 0):.4g} KB  WRITE_SIZE {m.get('WRITE_SIZE', 0):.4g} KB")
