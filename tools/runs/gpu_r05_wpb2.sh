#!/bin/bash
# Round 5: 2-wave workgroups (4 scenarios, four per CU) for config 2, possible only
# with TEMP outside LDS (FPF_WAVE_TEMP_VMEM in the per-plan build): the default
# command (two streams, K = 50) for the default, VMEM TEMP at 4-wave workgroups,
# and VMEM TEMP at 2-wave workgroups; the aggregate must agree. Two rounds.
set -o pipefail
OUT=gpurun_out/r05wpb2
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python3 -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c4 > $OUT/$n.log 2>&1 || { echo "FAILED $n"; tail -8 $OUT/$n.log; exit 1; }
  python3 -c "
import json
a=json.loads(open('$OUT/$n.log').read().strip().splitlines()[-1]); g=a['aggregate']
print('$n', round(a['value']/1e6,2), 'M/s', 'ms/step', round(a['ms_per_step']*1e3,2), 'us', 'kernel', round(a['roofline']['kernel_ms']*1e3,2), 'rtc', a['config']['wave_rtc_builds'], 'conv', g['n_conv'], 'loss', repr(g['loss_sum_kw']))"
}
for r in 1 2; do
  run def_r$r FPF_X=0 || exit 1
  run vm4_r$r FPF_WAVE_RTC_DEFS=FPF_WAVE_TEMP_VMEM,FPF_WAVE_TEMP_LATE || exit 1
  run vm2_r$r FPF_WAVE_RTC_DEFS=FPF_WAVE_TEMP_VMEM,FPF_WAVE_TEMP_LATE FPF_WAVE_WPB=2 || exit 1
done
