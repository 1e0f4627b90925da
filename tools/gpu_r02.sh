#!/bin/bash
# Round-2 measurement: the default bench line (config 2 + config-4 roofline +
# CPU baseline), then kernel-trace stats and FETCH_SIZE / WRITE_SIZE passes for
# configs 2, 4 and 3.  Every GPU step has its own time limit; the first failure
# ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${R:-r02}
timeout -k 10 400 python3 -u bench.py > gpurun_out/${R}_bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/${R}_bench.log; exit 1; }
tail -1 gpurun_out/${R}_bench.log
TAG=${R}_c2 tools/gpu_profile.sh || exit 1
TAG=${R}_c4 ARGS="--config 4 --steps 6 --warmup 2 --no-cpu-baseline" PARGS="--config 4 --steps 3 --warmup 1 --no-cpu-baseline" tools/gpu_profile.sh || exit 1
if [ -z "$SKIP_C3" ]; then
  TAG=${R}_c3 ARGS="--config 3 --steps 4 --warmup 1 --no-cpu-baseline" PARGS="--config 3 --steps 2 --warmup 1 --no-cpu-baseline" tools/gpu_profile.sh || exit 1
fi
echo DONE
