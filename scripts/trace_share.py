"""Share of a traced step by kernel class (the MFMA kernels vs the rest), from a kernel_stats_top
summary (profiles/*_kernel_stats_*.txt): python scripts/trace_share.py FILE"""
import re
import sys

MFMA = ("conv3x3_x3_kernel", "conv3x3_x3p_kernel", "wgrad3_kernel", "wgrad2_kernel", "wgrad_kernel", "gram_kernel",
        "gram_bwd_kernel", "gemm_kernel", "gemm_wide_kernel", "gemm_x3_kernel", "conv3x3_f32_kernel",
        "conv3x3_cin3_x3_kernel", "wgrad_co3_kernel", "gram_x3_kernel")  # round 6: split-bf16 cin <= 3 conv, cout <= 3 wgrad, Gram
VALU_CONV = ("conv3x3_cin4_kernel", "conv3x3_smallc", "wgrad_smallco_kernel")
tot = 0.0
cls = {"mfma": 0.0, "valu conv": 0.0, "other": 0.0}
other = []
for line in open(sys.argv[1]):
    m = re.match(r"\s+([\d.]+) ms\s+(\d+)x\s+([\d.]+) us\s+(.*)", line)
    if not m:
        continue
    ms, name = float(m.group(1)), m.group(4)
    tot += ms
    k = "mfma" if name.startswith(MFMA) else "valu conv" if name.startswith(VALU_CONV) else "other"
    cls[k] += ms
    if k == "other":
        other.append((ms, name))
for k, v in cls.items():
    print(f"{k:10s} {v:9.2f} ms  {v / tot:6.1%}")
print("largest others:", ", ".join(f"{n.split('<')[0]} {ms / tot:.1%}" for ms, n in sorted(other, reverse=True)[:8]))
