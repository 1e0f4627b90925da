"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin):
one line per kernel with VGPRs, spills, scratch, occupancy, LDS."""
import re
import sys

cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key, pat in (("vgpr", r" VGPRs: (\d+)"), ("spill", r"VGPRs Spill: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, line)
        if m:
            cur[key] = int(m.group(1))
for r in rows:
    name = r["name"]
    m = re.search(r"dpf_wave_kernelILi(\d+)ELi(\d+)ELb(\d)ELi(\d+)E", name)
    tag = f"wave spw{m.group(1)} C{m.group(2)} full{m.group(3)} wpb{m.group(4)}" if m else name[:60]
    print(f"{tag:40s} vgpr {r.get('vgpr')} spill {r.get('spill')} scratch {r.get('scratch')} occ {r.get('occ')} lds {r.get('lds')}")
