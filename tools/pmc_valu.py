"""Record the VALU instruction count per launch of a workload's dominant kernel
from an SQ counter pass (tools/runs/gpu_pmc_sq.sh, pass 1 holds SQ_INSTS_VALU) in
profiles/pmc_traffic.json, where bench.py's instruction-efficiency figure reads it:

    python tools/pmc_valu.py <sq-tag> "<workload>" <kernel-name-substring> [<profile tag>]
"""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag, workload, kname = sys.argv[1], sys.argv[2], sys.argv[3]
    ptag = sys.argv[4] if len(sys.argv) > 4 else tag
    path = os.path.join(ROOT, "gpurun_out", f"pmc_{tag}_1", "pmc_counter_collection.csv")
    per = defaultdict(float)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] == "SQ_INSTS_VALU" and kname in row["Kernel_Name"]:
            per[row["Dispatch_Id"]] += float(row["Counter_Value"])
    if not per:
        sys.exit(f"no SQ_INSTS_VALU rows for {kname} in {path}")
    v = sum(per.values()) / len(per)
    tp = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    d = json.load(open(tp))
    e = d["by_workload"].setdefault(workload, {})
    e["valu_insts_per_launch"] = v
    e["valu_tag"] = ptag
    json.dump(d, open(tp, "w"), indent=1)
    print(workload, kname, "VALU insts per launch", v, "over", len(per), "launches")


if __name__ == "__main__":
    main()
