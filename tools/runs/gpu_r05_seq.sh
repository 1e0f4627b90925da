#!/bin/bash
# Round 5: the sequential-order plan's GPU tests and its bench diagnostic leg
set -o pipefail
OUT=gpurun_out/r05seq
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_lag.py > $OUT/pytest.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAIL|Error" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python3 -u -c "
import json, torch, bench
dev = torch.device('cuda:0'); st = torch.cuda.current_stream()
print(json.dumps(bench._diag_sequential_order(torch, 0, st, dev)))
" > $OUT/diag.log 2>&1 || { echo "DIAG FAILED"; tail -30 $OUT/diag.log; exit 1; }
tail -1 $OUT/diag.log
