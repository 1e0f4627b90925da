#!/bin/bash
# Kernel time vs batch size on the 123-bus feeder (wave kernel): the latency of
# one wavefront's solve (B = 2) against full-chip batches.
set -o pipefail
mkdir -p gpurun_out/bsweep
for B in ${BS:-2 16 256 1024 4096 16384}; do
  timeout -k 10 200 python3 -u bench.py --scenarios $B --steps 20 --warmup 3 --no-cpu-baseline --no-c4 --in-batches 1 > gpurun_out/bsweep/b$B.log 2>&1 || { echo "FAILED $B"; tail -5 gpurun_out/bsweep/b$B.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/bsweep/b$B.log').read().strip().splitlines()[-1]); print('B $B kernel_ms %.4f ms_per_step %.4f' % (d['roofline']['kernel_ms'], d['ms_per_step']))"
done
