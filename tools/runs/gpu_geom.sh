#!/bin/bash
# Geometry sweep of the hipRTC-specialised kernel on the GPU box:
# GEOMS="nt,maxt,min_waves:tile ..." (FPF_RTC_GEOM diagnostic override).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for G in ${GEOMS:-512,1,4:4}; do
  GEO=${G%%:*}; T=${G##*:}
  if [ -n "$STAMPS" ]; then
    FPF_RTC_GEOM=$GEO TILE=$T timeout -k 10 200 python tools/stamps.py >> gpurun_out/geom_stamps.log 2>&1 || { echo "STAMPS FAILED $G"; tail gpurun_out/geom_stamps.log; exit 1; }
    tail -1 gpurun_out/geom_stamps.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('  stamps $G', {k: int(v) for k, v in d['mean_cycles'].items()})"
  fi
  FPF_RTC_GEOM=$GEO timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --tile $T > gpurun_out/geom_$T.log 2>&1 || { echo "BENCH FAILED $G"; tail -30 gpurun_out/geom_$T.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/geom_$T.log').read().strip().splitlines()[-1]); c=d['config']; print('$G','tile',c['tile'],'spec',c['specialized'],'value %.3e'%d['value'],'kern ms %.4f'%d['roofline']['kernel_ms'])"
done
