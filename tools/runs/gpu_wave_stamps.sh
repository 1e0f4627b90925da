#!/bin/bash
# Stage and in-sweep phase split of the wave kernel (stamps build) for each
# batch size in $BS (FPF_WAVE_GEOM from $GEOM if set).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in ${BS:-4096}; do
  B=$B timeout -k 10 180 python tools/wave_stamps.py > gpurun_out/wstamps_$B.log 2>&1 || { echo "STAMPS $B FAILED"; tail -20 gpurun_out/wstamps_$B.log; exit 1; }
  echo "B $B: $(tail -1 gpurun_out/wstamps_$B.log)"
done
