#!/bin/bash
# round 3: the paired kernel after the batched hand-off loads: its tests, the diagnostic leg
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r03k
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_wcoop.py -m gpu -x -q --timeout 150 --timeout-method thread > $D/pytest_wcoop.log 2>&1 || { echo "WCOOP TESTS FAILED"; tail -60 $D/pytest_wcoop.log; exit 1; }
tail -1 $D/pytest_wcoop.log
timeout -k 10 300 python3 -u -c "
import json, sys, torch
sys.path.insert(0, '.')
import bench
r = bench._diag_4096(torch, 0, torch.cuda.current_stream(0), torch.device('cuda', 0))
print(json.dumps(r))
" > $D/diag.log 2>&1 || { echo "DIAG FAILED"; tail -30 $D/diag.log; exit 1; }
tail -1 $D/diag.log
echo DONE
