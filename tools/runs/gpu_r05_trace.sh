#!/bin/bash
# the timed region's fixed costs (dist.timed_study, FPF_BENCH_TRACE)
set -o pipefail
OUT=gpurun_out/r05tr
mkdir -p $OUT
export TMPDIR=/tmp FPF_BENCH_TRACE=1
for S in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c4 --streams $S > $OUT/s$S.log 2> $OUT/s$S.err || { echo "FAILED S=$S"; tail -20 $OUT/s$S.err; exit 1; }
  grep timed_study $OUT/s$S.err
  python3 -c "
import json; d=json.loads([l for l in open('$OUT/s$S.log') if l.startswith('{')][-1])
print('S=$S value %.1f M/s ms_per_step %.4f kernel_ms(ev) %.4f' % (d['value']/1e6, d['ms_per_step'], d['roofline']['kernel_ms']))"
done
