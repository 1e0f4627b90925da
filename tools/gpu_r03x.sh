#!/bin/bash
# round 3 final evidence for the swizzled wave kernel: rocprofv3 stats + FETCH/WRITE
# passes for configs 2 and 4, and the SQ passes (tools/gpu_profile.sh, gpu_pmc_sq.sh)
set -o pipefail
export TMPDIR=/tmp
P=r03x
TAG=${P}_c2 ARGS="--steps 30 --warmup 5 --no-cpu-baseline --no-c4" bash tools/gpu_profile.sh || exit 1
TAG=${P}_c4 ARGS="--config 4 --steps 10 --warmup 2 --no-cpu-baseline" PARGS="--config 4 --steps 5 --warmup 1 --no-cpu-baseline" bash tools/gpu_profile.sh || exit 1
TAG=${P}_sq_c2 ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-c4" bash tools/gpu_pmc_sq.sh > gpurun_out/${P}_sq_c2.txt || exit 1
TAG=${P}_sq_c4 ARGS="--config 4 --steps 3 --warmup 1 --no-cpu-baseline" bash tools/gpu_pmc_sq.sh > gpurun_out/${P}_sq_c4.txt || exit 1
for c in c2 c4; do echo "== $c"; grep -E "wave" gpurun_out/prof_${P}_$c/trace_kernel_stats.csv | cut -d, -f1-4; done
echo DONE
