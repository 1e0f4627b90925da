#!/bin/bash
# Round 5: the default bench command at 2 and 3 streams (config 2, K = 50), alternating, three rounds.
set -o pipefail
OUT=gpurun_out/r05st3s
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3; do
for S in 2 3; do
  timeout -k 10 200 python3 -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c4 --streams $S > $OUT/s${S}_r$r.log 2>&1 || { echo "FAILED $S"; tail -5 $OUT/s${S}_r$r.log; exit 1; }
  python3 -c "
import json
a=json.loads(open('$OUT/s${S}_r$r.log').read().strip().splitlines()[-1])
print('streams $S r$r', round(a['value']/1e6,2), 'M/s', 'ms/step', round(a['ms_per_step']*1e3,2), 'us', 'kernel', round(a['roofline']['kernel_ms']*1e3,2))"
done
done
