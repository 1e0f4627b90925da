#!/bin/bash
# Round 6, second session: the host-synchronous VVC round with the staged step-size
# search (fpf_vvc.cpp: vvc_line_search, lazy 32): the VVC GPU tests and the leg
set -o pipefail
P=${P:-r06s2_vvc2}
mkdir -p gpurun_out/$P
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -k "vvc or integration" -q --timeout 200 --timeout-method thread > gpurun_out/$P/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/$P/pytest.log; exit 1; }
tail -1 gpurun_out/$P/pytest.log
for r in 1 2; do
  timeout -k 10 200 python3 -u tools/vvc_round_leg.py > gpurun_out/$P/leg_$r.log 2>&1 || { tail -20 gpurun_out/$P/leg_$r.log; exit 1; }
  grep best gpurun_out/$P/leg_$r.log
done
echo DONE
