"""Summarise a gpu_profile.sh run into profiles/<tag>/:

    python tools/pmc_summary.py <tag> [kernel-name-substring] [run-dir]

(run-dir: a tools/runs/gpu_wblk.sh-style directory holding prof/run_kernel_stats.csv,
pmc_<COUNTER>/pmc_counter_collection.csv and the bench line bench_*.json;
default: the gpu_profile.sh layout gpurun_out/prof_<tag>...)

Copies the rocprofv3 kernel stats, and turns the separate FETCH_SIZE and
WRITE_SIZE passes into per-launch HBM bytes of the dominant kernel, corrected
as MI355X_MICROARCH.md section HBM prescribes: FETCH_SIZE (KiB) reports half
the bytes of a wide coalesced read on gfx950, so it is doubled; WRITE_SIZE
(KiB) is taken as is.  Writes profiles/<tag>/pmc.json and refreshes this
workload's entry of profiles/pmc_traffic.json ({"by_workload": {"123-bus x
4096": {...}, ...}}), which bench.py reads for roofline.traffic.
"""
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path, counter, kname):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter and kname in row["Kernel_Name"]:
                vals.append(float(row["Counter_Value"]))
    return vals


def main():
    tag = sys.argv[1]
    kname = sys.argv[2] if len(sys.argv) > 2 else "fpf_rtc_tiled"
    out = os.path.join(ROOT, "gpurun_out")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    if len(sys.argv) > 3:
        run = sys.argv[3]
        shutil.copy(os.path.join(run, "prof", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
        bfile = sorted(f for f in os.listdir(run) if f.startswith("bench") and f.endswith(".json"))[0]
        bench = [ln for ln in open(os.path.join(run, bfile)) if ln.startswith("{")]
        pmc = lambda c: os.path.join(run, f"pmc_{c}", "pmc_counter_collection.csv")
    else:
        shutil.copy(os.path.join(out, f"prof_{tag}", "trace_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
        bench = [ln for ln in open(os.path.join(out, f"prof_{tag}_bench.log")) if ln.startswith("{")]
        pmc = lambda c: os.path.join(out, f"pmc_{tag}_{c}", "pmc_counter_collection.csv")
    fetch = per_launch(pmc("FETCH_SIZE"), "FETCH_SIZE", kname)
    write = per_launch(pmc("WRITE_SIZE"), "WRITE_SIZE", kname)
    b = json.loads(bench[-1]) if bench else {}
    fk = sum(fetch) / len(fetch)
    wk = sum(write) / len(write)
    hbm = (2 * fk + wk) * 1024
    with open(os.path.join(dst, "kernel_stats.csv")) as f:
        avg_ns = next(float(r["AverageNs"]) for r in csv.DictReader(f) if kname in r["Name"])
    scen = b.get("config", {}).get("scenarios_per_gpu")
    m = re.search(r"(\d+)-bus", b.get("metric", ""))
    workload = f"{m.group(1) if m else 123}-bus x {scen}"
    res = {
        "tag": tag, "kernel": kname, "launches_fetch": len(fetch), "launches_write": len(write),
        "FETCH_SIZE_KiB_per_launch": fk, "WRITE_SIZE_KiB_per_launch": wk,
        "hbm_bytes_per_launch": hbm, "correction": "2 x FETCH_SIZE + WRITE_SIZE (gfx950, MI355X_MICROARCH.md HBM)",
        "rocprof_avg_kernel_ns": avg_ns, "bench_kernel_ms": b.get("roofline", {}).get("kernel_ms"),
        "bytes_alg_per_launch": (b.get("roofline", {}).get("bytes_alg_per_scenario") or 0) * (scen or 0),
        "workload": workload,
        "bench_line": b,
    }
    json.dump(res, open(os.path.join(dst, "pmc.json"), "w"), indent=1)
    tp = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(tp))
    except (OSError, ValueError):
        d = {}
    if "by_workload" not in d:   # the one-workload layout of round 1
        d = {"by_workload": {d["workload"]: d} if "workload" in d else {}}
    d["by_workload"][workload] = {k: res[k] for k in ("tag", "kernel", "hbm_bytes_per_launch", "bytes_alg_per_launch",
                                                     "rocprof_avg_kernel_ns", "bench_kernel_ms")}
    json.dump(d, open(tp, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "bench_line"}, indent=1))


if __name__ == "__main__":
    main()
