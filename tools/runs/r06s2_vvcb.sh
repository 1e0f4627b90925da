#!/bin/bash
# Round 6, second session: where the batched VVC rounds' time goes (kernel trace)
set -o pipefail
P=${P:-r06s2_vvcb}
mkdir -p gpurun_out/$P
export TMPDIR=/tmp
for F in demo dl_new 123bus; do
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/$P/kt_$F -o kt --output-format csv -- python3 tools/vvc_batch_leg.py $F 64 > gpurun_out/$P/leg_$F.log 2>&1 || { tail -20 gpurun_out/$P/leg_$F.log; exit 1; }
  grep feeder gpurun_out/$P/leg_$F.log
done
echo DONE
