#!/bin/bash
# round 3: where the config-5 multi-area solve spends its time (kernel + copy trace)
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r03n
mkdir -p $D
timeout -k 10 200 python3 -u tools/c5_leg.py > $D/c5.log 2>&1 || { echo "C5 FAILED"; tail -20 $D/c5.log; exit 1; }
tail -1 $D/c5.log
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o c5 -- python3 $GRAFT_REPO_ROOT/tools/c5_leg.py > $GRAFT_REPO_ROOT/$D/prof.log 2>&1 || { echo "PROF FAILED"; tail -20 $GRAFT_REPO_ROOT/$D/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
find $D/prof -name "*.csv" | head
echo DONE
