#!/bin/bash
# Round 5: config 2 (one wave round, two 4-wave workgroups per CU) with the second
# resident workgroup of each CU started late (FPF_WAVE_WG_STAGGER=lo,hi,n: n x ~1 k
# cycles), so the first one's loads land, and its V leaves, without the second's
# competing for HBM.  Per-plan builds on (default).
set -o pipefail
OUT=gpurun_out/r05hstag
mkdir -p $OUT
export TMPDIR=/tmp
STAGS=${STAGS:-"0,0,0 256,512,3 256,512,6 256,512,9 256,512,12"}
for r in 1 2; do
for S in $STAGS; do
  T=${S//,/_}
  FPF_WAVE_WG_STAGGER=$S timeout -k 10 200 python3 -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-c4 --streams 1 > $OUT/s_${T}_r$r.log 2>&1 || { echo "FAILED $S"; tail -5 $OUT/s_${T}_r$r.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/s_${T}_r$r.log').read().strip().splitlines()[-1])
print('$S r$r', 'c2 us', round(d['roofline']['kernel_ms']*1e3,2), 'value', round(d['value']/1e6,1), 'n_conv', d['aggregate']['n_conv'], 'rtc', d['config']['wave_rtc_builds'])"
done
done
