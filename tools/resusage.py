"""Tabulate -Rpass-analysis=kernel-resource-usage remarks (VGPRs, AGPRs, spills, scratch,
occupancy, LDS) per kernel.  usage: python tools/resusage.py LOG [substring ...]"""
import re
import sys

txt = open(sys.argv[1]).read().split("Function Name: ")
keys = [("VGPRs", r"VGPRs: (\d+)"), ("AGPRs", r"AGPRs: (\d+)"), ("spill", r"VGPRs Spill: (\d+)"),
        ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"),
        ("lds", r"LDS Size \[bytes/block\]: (\d+)")]
for blk in txt[1:]:
    name = blk.split()[0]
    if len(sys.argv) > 2 and not any(s in name for s in sys.argv[2:]):
        continue
    vals = []
    for k, pat in keys:
        m = re.search(pat, blk)
        vals.append(f"{k} {m.group(1) if m else '?'}")
    print(f"{name[:70]:70s} " + "  ".join(vals))
