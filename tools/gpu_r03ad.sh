#!/bin/bash
# the paired kernel's stage split (stamps build), then the whole GPU suite and smoke
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r03ad
mkdir -p $D
timeout -k 10 200 python -u tools/coop_stamps.py > $D/stamps.log 2>&1 || { echo "STAMPS FAILED"; tail -20 $D/stamps.log; }
tail -1 $D/stamps.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { echo "GPU SUITE FAILED"; tail -60 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $D/smoke.log; exit 1; }
tail -3 $D/smoke.log
echo DONE
