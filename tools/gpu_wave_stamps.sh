#!/bin/bash
# Stage split of the wave kernel (stamps build) for each FPF_WAVE_GEOM in $GEOMS.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for G in ${GEOMS:-2,4}; do
  FPF_WAVE_GEOM=$G timeout -k 10 120 python tools/wave_stamps.py > gpurun_out/wstamps_$G.log 2>&1 || { echo "STAMPS $G FAILED"; tail -20 gpurun_out/wstamps_$G.log; exit 1; }
  echo "geom $G: $(tail -1 gpurun_out/wstamps_$G.log)"
done
