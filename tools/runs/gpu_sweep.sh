#!/bin/bash
# Kernel-variant sweep on the GPU box: SWEEP="ENV=VAL+ENV2=VAL2 ..." -- each item
# a set of fpf_feeder_create knobs (FPF_RTC_TRACKS, FPF_RTC_AHEAD, FPF_RTC_GEOM,
# FPF_RTC_SCHEDBAR); one short bench per item.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for ITEM in ${SWEEP:-DEFAULT=1}; do
  i=$((i+1))
  ENVS=$(echo "$ITEM" | tr '+' ' ')
  env $ENVS timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/sweep_$i.log 2>&1 || { echo "BENCH FAILED $ITEM"; tail -20 gpurun_out/sweep_$i.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/sweep_$i.log') if l.startswith('{')][-1]); r=d['roofline']; print('$ITEM', 'value %.4e' % d['value'], 'kern_us %.2f' % (r['kernel_ms']*1e3), 'frac %.4f' % r['frac'], 'ms/step %.4f' % d['ms_per_step'])"
done
