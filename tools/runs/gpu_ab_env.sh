#!/bin/bash
# Same-box A/B of the wave kernel's variants: for each "tag:ENV=.. ENV2=.." in
# $VARIANTS, the config-4 roofline leg and config 2 (both layouts) kernel times.
# Example: VARIANTS="base:FPF_WAVE_PERSIST=0 per:FPF_WAVE_PERSIST=1" bash tools/runs/gpu_ab_env.sh
set -o pipefail
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in ${REPS:-1 2}; do
for V in $VARIANTS; do
  name=${V%%:*}; envs=${V#*:}; envs=${envs//,/ }
  for cfg in ${CFGS:-"4:1" "2:1" "2:0"}; do
    c=${cfg%%:*}; lay=${cfg#*:}
    log=$OUT/${name}_c${c}_l${lay}_r${rep}.log
    extra=""; [ "$c" = "2" ] && extra="--no-c4"
    env $envs timeout -k 10 300 python -u bench.py --config $c --layout $lay --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline $extra > $log 2>&1 || { echo "FAILED $name c$c l$lay"; tail -20 $log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$log').read().strip().splitlines()[-1])
r=d['roofline']; print('$name', 'c$c', 'l$lay', 'r$rep', 'kernel_ms', round(r['kernel_ms'],5), 'frac', round(r['frac'],4), 'n_conv', d['aggregate']['n_conv'])"
  done
done
done
