#!/bin/bash
# Round 5: config 2 with the steps on 1, 2 and 4 HIP streams (independent batches)
set -o pipefail
OUT=gpurun_out/r05st
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
for S in 1 2 4; do
  timeout -k 10 300 python3 -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-c4 --streams $S > $OUT/s${S}_r$rep.log 2>&1 || { echo "FAILED S=$S"; tail -20 $OUT/s${S}_r$rep.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$OUT/s${S}_r$rep.log') if l.startswith('{')][-1])
print('S=$S r$rep value %.1f M/s ms_per_step %.4f kernel_ms(ev) %.4f n_conv %d rtc %d' % (d['value']/1e6, d['ms_per_step'], d['roofline']['kernel_ms'], d['aggregate']['n_conv'], d['config']['wave_rtc_builds']))"
done
done
