#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/geom
for G in "2,4" "1,2" "1,4"; do
  FPF_WAVE_GEOM=$G timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/geom/g_${G/,/_}.log 2>&1 || { echo "FAILED $G"; tail -5 gpurun_out/geom/g_${G/,/_}.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/geom/g_${G/,/_}.log').read().strip().splitlines()[-1])
print('$G', 'c2 ms', round(d['roofline']['kernel_ms'],4), 'c4 ms', round(d['roofline_config4']['kernel_ms'],4), 'n_conv', d['aggregate']['n_conv'])"
done
