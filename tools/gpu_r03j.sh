#!/bin/bash
# round 3: the paired kernel's diagnostic leg (bench) and its rocprof stats
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r03j
mkdir -p $D
timeout -k 10 300 python3 -u -c "
import json, sys, torch
sys.path.insert(0, '.')
import bench
r = bench._diag_4096(torch, 0, torch.cuda.current_stream(0), torch.device('cuda', 0))
print(json.dumps(r))
" > $D/diag.log 2>&1 || { echo "DIAG FAILED"; tail -30 $D/diag.log; exit 1; }
tail -1 $D/diag.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o prof -- python3 -u -c "
import json, sys, torch
sys.path.insert(0, '$GRAFT_REPO_ROOT')
import bench
r = bench._diag_4096(torch, 0, torch.cuda.current_stream(0), torch.device('cuda', 0))
print(json.dumps(r))
" > $GRAFT_REPO_ROOT/$D/prof.log 2>&1 || { echo "PROF FAILED"; tail -30 $GRAFT_REPO_ROOT/$D/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
find $D/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c "cut -d, -f1-4 {} | head -8"
echo DONE
