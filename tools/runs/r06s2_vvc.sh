#!/bin/bash
# Round 6, second session: where a config-1 host-synchronous VVC round's time goes
set -o pipefail
P=${P:-r06s2_vvc}
mkdir -p gpurun_out/$P
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/vvc_round_leg.py > gpurun_out/$P/leg.log 2>&1 || { tail -20 gpurun_out/$P/leg.log; exit 1; }
cat gpurun_out/$P/leg.log | grep best
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --runtime-trace -d gpurun_out/$P/kt -o kt --output-format csv -- python3 tools/vvc_round_leg.py > gpurun_out/$P/kt.log 2>&1 || { tail -20 gpurun_out/$P/kt.log; exit 1; }
ls gpurun_out/$P/kt
echo DONE
