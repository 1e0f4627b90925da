#!/bin/bash
# round 3 final evidence for the wave and wave-block kernels: rocprofv3 stats +
# FETCH/WRITE passes for configs 2, 4, 3 and the SQ passes (tools/gpu_r03e.sh)
set -o pipefail
export TMPDIR=/tmp
P=r03q bash tools/gpu_r03e.sh || exit 1
echo DONE
