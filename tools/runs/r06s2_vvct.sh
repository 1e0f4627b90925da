#!/bin/bash
# Round 6, second session: the host-synchronous VVC round's stages (FPF_VVC_TRACE)
set -o pipefail
P=${P:-r06s2_vvct}
mkdir -p gpurun_out/$P
export TMPDIR=/tmp
FPF_VVC_TRACE=1 timeout -k 10 200 python3 -u tools/vvc_round_leg.py > gpurun_out/$P/leg.log 2> gpurun_out/$P/trace.log || { tail -20 gpurun_out/$P/trace.log; exit 1; }
cat gpurun_out/$P/leg.log | grep best
tail -12 gpurun_out/$P/trace.log
echo DONE
