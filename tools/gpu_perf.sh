#!/bin/bash
# Perf iteration on the GPU box: stamp split + bench at several tiles + rocprof stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for T in ${TILES:-0}; do
  TILE=$T timeout -k 10 200 python tools/stamps.py >> gpurun_out/stamps.log 2>&1 || { echo "STAMPS FAILED"; tail gpurun_out/stamps.log; exit 1; }
done
cat gpurun_out/stamps.log | grep '^{'
for T in ${TILES:-0}; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --tile $T > gpurun_out/bench_t$T.log 2>&1 || { echo "BENCH FAILED"; tail gpurun_out/bench_t$T.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_t$T.log').read().strip().splitlines()[-1]); print('tile',d['config']['tile'],'value %.3e'%d['value'],'ms/step %.4f'%d['ms_per_step'],'kern ms %.4f'%d['roofline']['kernel_ms'],'frac %.3f'%d['roofline']['frac'])"
done
