#!/bin/bash
# round 3: zeroed phases on the paired kernel: its tests, the diagnostic leg
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r03y
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_wcoop.py -m gpu -x -v --timeout 200 --timeout-method thread > $D/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -60 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
timeout -k 10 300 python3 -u -c "
import json, sys, torch
sys.path.insert(0, '.')
import bench
r = bench._diag_4096(torch, 0, torch.cuda.current_stream(0), torch.device('cuda', 0))
print(json.dumps({k: r[k] for k in ('kernel_ms', 'speedup_vs_exact', 'iters_equal_exact', 'max_v_rel_diff_vs_exact')}))
" > $D/diag.log 2>&1 || { echo "DIAG FAILED"; tail -30 $D/diag.log; exit 1; }
tail -1 $D/diag.log
echo DONE
