#!/bin/bash
# Round 5: the default command (two streams, K = 50) with 4-wave (default) and
# 8-wave workgroups (FPF_WAVE_WPB=8) for config 2, alternating, three rounds.
set -o pipefail
OUT=gpurun_out/r05wpb2s
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3; do
for W in 4 8; do
  FPF_WAVE_WPB=$W timeout -k 10 200 python3 -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c4 > $OUT/w${W}_r$r.log 2>&1 || { echo "FAILED $W"; tail -5 $OUT/w${W}_r$r.log; exit 1; }
  python3 -c "
import json
a=json.loads(open('$OUT/w${W}_r$r.log').read().strip().splitlines()[-1])
print('wpb $W r$r', round(a['value']/1e6,2), 'M/s', 'ms/step', round(a['ms_per_step']*1e3,2), 'us', 'kernel', round(a['roofline']['kernel_ms']*1e3,2), 'rtc', a['config']['wave_rtc_builds'])"
done
done
