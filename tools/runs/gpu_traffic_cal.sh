#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (tools/ubench/traffic_cal): timing run,
# then one rocprofv3 --pmc pass per counter, per access pattern.
set -o pipefail
mkdir -p gpurun_out/cal
export TMPDIR=/tmp
for K in rd8 rd16 wr8 wr16 rd8s; do
  timeout -k 10 60 tools/ubench/traffic_cal $K 5 > gpurun_out/cal/$K.json || { echo "RUN $K FAILED"; exit 1; }
  cat gpurun_out/cal/$K.json
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $C -d gpurun_out/cal/pmc_${K}_$C -o pmc --output-format csv -- tools/ubench/traffic_cal $K 2 > gpurun_out/cal/pmc_${K}_$C.log 2>&1 || { echo "PMC $K $C FAILED"; tail -5 gpurun_out/cal/pmc_${K}_$C.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, json, glob
out = {}
for K in ["rd8", "rd16", "wr8", "wr16", "rd8s"]:
    b = json.load(open(f"gpurun_out/cal/{K}.json"))
    r = {"bytes": b["bytes_per_launch"], "GBps": b["GBps"]}
    for C in ["FETCH_SIZE", "WRITE_SIZE"]:
        vals = [float(row["Counter_Value"]) for row in csv.DictReader(open(f"gpurun_out/cal/pmc_{K}_{C}/pmc_counter_collection.csv"))
                if row["Counter_Name"] == C]
        r[C + "_KiB_per_launch"] = sum(vals) / len(vals) if vals else None
        r[C + "_bytes_ratio"] = (sum(vals) / len(vals) * 1024 / b["bytes_per_launch"]) if vals else None
    out[K] = r
print(json.dumps(out, indent=1))
json.dump(out, open("gpurun_out/cal/summary.json", "w"), indent=1)
PY
