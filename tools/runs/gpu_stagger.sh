#!/bin/bash
# Config-4 kernel time under workgroup start staggers (FPF_WAVE_WG_STAGGER=lo,hi,n).
set -o pipefail
mkdir -p gpurun_out/stag
STAGS=${STAGS:-"0,0,0 256,512,3 256,512,6 0,0,0"}
for S in $STAGS; do
  T=${S//,/_}
  FPF_WAVE_WG_STAGGER=$S timeout -k 10 200 python3 -u bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/stag/s_$T.log 2>&1 || { echo "FAILED $S"; tail -5 gpurun_out/stag/s_$T.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/stag/s_$T.log').read().strip().splitlines()[-1])
print('$S', 'c4 ms', round(d['roofline']['kernel_ms'],4), 'n_conv', d['aggregate']['n_conv'])"
done
