#!/bin/bash
# Round 5: FPF_WAVE_GROUP=2 (the next slot's Sld / TEMP reads issued before this slot's arithmetic) in the per-plan build:
# static kernel (tests/test_gpu_wave.py), then configs 2 and 4, two alternating rounds.
set -o pipefail
OUT=gpurun_out/r05grp
mkdir -p $OUT
export TMPDIR=/tmp
VARS=${VARS:-"base FPF_WAVE_GROUP=2"}
for V in $VARS; do
  D=$V; [ "$V" = base ] && D=""
  FPF_WAVE_RTC_DEFS=$D timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread "tests/test_gpu_wave.py::test_specialised_build_matches_static" > $OUT/eq_${V//,/+}.log 2>&1 || { echo "EQ FAILED $V"; tail -20 $OUT/eq_${V//,/+}.log; exit 1; }
  echo "eq $V: $(tail -1 $OUT/eq_${V//,/+}.log)"
done
for r in 1 2 3; do
for V in $VARS; do
  D=$V; [ "$V" = base ] && D=""
  T=${V//,/+}
  FPF_WAVE_RTC_DEFS=$D timeout -k 10 200 python3 -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-c4 --streams 1 > $OUT/c2_${T}_r$r.log 2>&1 || { echo "C2 FAILED $V"; tail -5 $OUT/c2_${T}_r$r.log; exit 1; }
  FPF_WAVE_RTC_DEFS=$D timeout -k 10 200 python3 -u bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/c4_${T}_r$r.log 2>&1 || { echo "C4 FAILED $V"; tail -5 $OUT/c4_${T}_r$r.log; exit 1; }
  python3 -c "
import json
a=json.loads(open('$OUT/c2_${T}_r$r.log').read().strip().splitlines()[-1]); b=json.loads(open('$OUT/c4_${T}_r$r.log').read().strip().splitlines()[-1])
print('$V r$r', 'c2 us', round(a['roofline']['kernel_ms']*1e3,2), 'c4 ms', round(b['roofline']['kernel_ms'],4), 'rtc', a['config']['wave_rtc_builds'], b['config']['wave_rtc_builds'], 'conv', a['aggregate']['n_conv'], b['aggregate']['n_conv'])"
done
done
