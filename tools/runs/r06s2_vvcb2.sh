#!/bin/bash
# Round 6, second session: the VVC batch paths on cached scratch (fpf::feeder_buf):
# the VVC GPU tests, then the batched-round leg per config-1 feeder
set -o pipefail
P=${P:-r06s2_vvcb2}
mkdir -p gpurun_out/$P
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -k "vvc or integration" -q --timeout 200 --timeout-method thread > gpurun_out/$P/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/$P/pytest.log; exit 1; }
tail -1 gpurun_out/$P/pytest.log
for F in demo dl_new 123bus; do
  timeout -k 10 200 python3 -u tools/vvc_batch_leg.py $F 64 > gpurun_out/$P/leg_$F.log 2>&1 || { tail -20 gpurun_out/$P/leg_$F.log; exit 1; }
  grep feeder gpurun_out/$P/leg_$F.log
done
echo DONE
