#!/bin/bash
# Round evidence (tag $P, default r02g): smoke, the GPU suite, the default bench line (config 2 + config-4 leg + copy
# check + host path + config-1 VVC round + CPU baseline), config 3 with its CPU
# baseline, then rocprofv3 stats + FETCH/WRITE passes for configs 2, 4 and 3.
set -o pipefail
P=${P:-r02g}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${P}_smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/${P}_smoke.log; exit 1; }
tail -3 gpurun_out/${P}_smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/${P}_pytest_gpu.log 2>&1 || { echo "GPU SUITE FAILED"; tail -30 gpurun_out/${P}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${P}_pytest_gpu.log
timeout -k 10 500 python3 -u bench.py > gpurun_out/${P}_bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/${P}_bench.log; exit 1; }
tail -1 gpurun_out/${P}_bench.log | cut -c1-300
timeout -k 10 500 python3 -u bench.py --config 3 --steps 5 --warmup 1 > gpurun_out/${P}_bench_c3.log 2>&1 || { echo "C3 FAILED"; tail -30 gpurun_out/${P}_bench_c3.log; exit 1; }
tail -1 gpurun_out/${P}_bench_c3.log | cut -c1-300
TAG=${P}_c2 ARGS="--steps 30 --warmup 5 --no-cpu-baseline --no-c4" bash tools/runs/gpu_profile.sh || exit 1
TAG=${P}_c4 ARGS="--config 4 --steps 10 --warmup 2 --no-cpu-baseline" PARGS="--config 4 --steps 5 --warmup 1 --no-cpu-baseline" bash tools/runs/gpu_profile.sh || exit 1
TAG=${P}_c3 ARGS="--config 3 --steps 5 --warmup 1 --no-cpu-baseline" PARGS="--config 3 --steps 3 --warmup 1 --no-cpu-baseline" bash tools/runs/gpu_profile.sh || exit 1
echo DONE
