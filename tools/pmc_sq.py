"""Per-dispatch means of the SQ counters collected by tools/runs/gpu_pmc_sq.sh, per
kernel (names containing 'fpf' or 'dpf'), plus per-wave ratios."""
import csv
import glob
import sys
from collections import defaultdict

tag = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [per dispatch]
for path in sorted(glob.glob(f"gpurun_out/pmc_{tag}_*/pmc_counter_collection.csv")):
    per = defaultdict(float)
    for row in csv.DictReader(open(path)):
        k = row["Kernel_Name"]
        if "fpf" not in k and "dpf" not in k:
            continue
        per[(k.split("(")[0], row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (k, d, c), v in per.items():
        vals[k][c].append(v)
for k, cs in vals.items():
    print(k)
    mean = {c: sum(v) / len(v) for c, v in cs.items()}
    waves = mean.get("SQ_WAVES")
    for c in sorted(mean):
        extra = f"   per wave {mean[c] / waves:12.1f}" if waves and c != "SQ_WAVES" else ""
        print(f"  {c:28s} {mean[c]:16.1f}  (n={len(cs[c])}){extra}")
