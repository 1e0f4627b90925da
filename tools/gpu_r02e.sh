#!/bin/bash
# Round-2 (r02e) evidence: the default bench line (config 2 + config-4 leg + copy
# check + host path + config-1 VVC round + CPU baseline), config 3 with its CPU
# baseline, then rocprofv3 stats + FETCH/WRITE passes for configs 2, 4 and 3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python3 -u bench.py > gpurun_out/r02e_bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/r02e_bench.log; exit 1; }
tail -1 gpurun_out/r02e_bench.log | cut -c1-300
timeout -k 10 500 python3 -u bench.py --config 3 --steps 5 --warmup 1 > gpurun_out/r02e_bench_c3.log 2>&1 || { echo "C3 FAILED"; tail -30 gpurun_out/r02e_bench_c3.log; exit 1; }
tail -1 gpurun_out/r02e_bench_c3.log | cut -c1-300
TAG=r02e_c2 ARGS="--steps 30 --warmup 5 --no-cpu-baseline --no-c4" bash tools/gpu_profile.sh || exit 1
TAG=r02e_c4 ARGS="--config 4 --steps 10 --warmup 2 --no-cpu-baseline" PARGS="--config 4 --steps 5 --warmup 1 --no-cpu-baseline" bash tools/gpu_profile.sh || exit 1
TAG=r02e_c3 ARGS="--config 3 --steps 5 --warmup 1 --no-cpu-baseline" PARGS="--config 3 --steps 3 --warmup 1 --no-cpu-baseline" bash tools/gpu_profile.sh || exit 1
echo DONE
