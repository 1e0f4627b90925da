#!/bin/bash
# Perf iteration on the GPU box: bench at several tiles, hipRTC-specialised and
# interpreted (optional stamp split of the interpreted kernel with STAMPS=1).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$STAMPS" ]; then
  for T in ${TILES:-0}; do
    TILE=$T timeout -k 10 200 python tools/stamps.py >> gpurun_out/stamps.log 2>&1 || { echo "STAMPS FAILED"; tail gpurun_out/stamps.log; exit 1; }
  done
  grep '^{' gpurun_out/stamps.log
fi
for V in ${VARIANTS:-rtc interp}; do
  for T in ${TILES:-0}; do
    EXTRA=""; [ "$V" = "interp" ] && EXTRA="--no-specialize"
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --tile $T $EXTRA > gpurun_out/bench_${V}_t$T.log 2>&1 || { echo "BENCH FAILED $V $T"; tail -30 gpurun_out/bench_${V}_t$T.log; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/bench_${V}_t$T.log').read().strip().splitlines()[-1]); c=d['config']; print('$V','tile',c['tile'],'spec',c['specialized'],'value %.3e'%d['value'],'ms/step %.4f'%d['ms_per_step'],'kern ms %.4f'%d['roofline']['kernel_ms'],'frac %.4f'%d['roofline']['frac'])"
  done
done
