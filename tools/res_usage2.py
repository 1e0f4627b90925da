"""Per-kernel VGPRs / spills / occupancy from `hipcc -Rpass-analysis=kernel-resource-usage` output (stdin).

    hipcc ... -Rpass-analysis=kernel-resource-usage -c x.hip 2>&1 | python tools/res_usage2.py [filter]
"""
import re
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"remark: +Function Name: (\S+)", line) or re.search(r"remark: +Name: (\S+)", line)
    if m and "Name:" in line and "Kernel" not in line:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark: +(VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]|ScratchSize \[bytes/lane\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split(" [")[0]] = int(m.group(2))
for r in rows:
    if flt in r["name"]:
        print(f"{r['name'][:70]:72s} vgpr={r.get('VGPRs')} agpr={r.get('AGPRs')} vspill={r.get('VGPRs Spill')} "
              f"sspill={r.get('SGPRs Spill')} occ={r.get('Occupancy')} scratch={r.get('ScratchSize')}")
