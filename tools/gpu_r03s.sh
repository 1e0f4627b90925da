#!/bin/bash
# round 3: the heavy mixed-load diagnostic leg (configs 2 and 3 at full size) alone
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r03s
mkdir -p $D
timeout -k 10 400 python3 -u -c "
import json, sys, torch
sys.path.insert(0, '.')
import bench
print(json.dumps(bench._diag_heavy(torch, 0, torch.cuda.current_stream(0), torch.device('cuda', 0)), indent=1))
" > $D/heavy.log 2>&1 || { echo "HEAVY FAILED"; tail -30 $D/heavy.log; exit 1; }
cat $D/heavy.log | tail -40
echo DONE
