#!/bin/bash
# Round-6 SQ passes: configs 2, 4 and 3 on the product kernels; config 3 again with
# the wave-block per-plan build's block offsets one block per thread instead of one
# (block, phase) per thread (FPF_WAVE_WBLK_NO_OFF3: the bank-conflict A/B) and its
# kernel time beside the product's.
set -o pipefail
export TMPDIR=/tmp
TAG=r06_c2 ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-c4 --streams 1" bash tools/runs/gpu_pmc_sq.sh || exit 1
TAG=r06_c4 ARGS="--config 4 --steps 3 --warmup 1 --no-cpu-baseline --streams 1" bash tools/runs/gpu_pmc_sq.sh || exit 1
TAG=r06_c3 ARGS="--config 3 --steps 2 --warmup 1 --no-cpu-baseline --streams 1" bash tools/runs/gpu_pmc_sq.sh || exit 1
FPF_WAVE_RTC_DEFS=FPF_WAVE_WBLK_NO_OFF3 TAG=r06_c3nooff3 ARGS="--config 3 --steps 2 --warmup 1 --no-cpu-baseline --streams 1" bash tools/runs/gpu_pmc_sq.sh || exit 1
mkdir -p gpurun_out/r06_off3
for v in off3 nooff3 off3b nooff3b; do
  D=""; case $v in nooff3*) D=FPF_WAVE_WBLK_NO_OFF3 ;; esac
  FPF_WAVE_RTC_DEFS=$D timeout -k 10 300 python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline --streams 1 > gpurun_out/r06_off3/c3_$v.json 2>&1 || { echo "C3 FAILED $v"; tail -5 gpurun_out/r06_off3/c3_$v.json; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r06_off3/c3_$v.json').readlines()[-1]); print('c3 $v', round(d['roofline']['kernel_ms'],4), 'ms')"
done
echo DONE
