#!/bin/bash
# The default bench line (config 2 + config-4 roofline + copy check + host path
# + config-1 VVC round + CPU baseline), then config 3 with its CPU baseline.
set -o pipefail
mkdir -p gpurun_out
R=${R:-r02c}
timeout -k 10 400 python3 -u bench.py > gpurun_out/${R}_bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/${R}_bench.log; exit 1; }
tail -1 gpurun_out/${R}_bench.log | cut -c1-400
if [ -z "$SKIP_C3" ]; then
  timeout -k 10 600 python3 -u bench.py --config 3 --steps 3 --warmup 1 > gpurun_out/${R}_bench_c3.log 2>&1 || { echo "C3 FAILED"; tail -30 gpurun_out/${R}_bench_c3.log; exit 1; }
  tail -1 gpurun_out/${R}_bench_c3.log | cut -c1-400
fi
