#!/bin/bash
# round 3 final: the default bench line (all legs, CPU baseline) and the rocprof
# stats of the paired kernel's diagnostic leg
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r03r
mkdir -p $D
timeout -k 10 700 python3 -u bench.py > $D/bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 $D/bench.log; exit 1; }
tail -1 $D/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'c2', d['roofline']['kernel_ms'], d['roofline']['frac'], 'c4', d['roofline_config4']['kernel_ms'], d['roofline_config4']['frac'], 'c3', d['roofline_config3']['kernel_ms'], d['roofline_config3']['frac']); print(json.dumps(d.get('diag_4096bus'))); print(json.dumps(d.get('config5_areas'))); print(json.dumps(d.get('cpu_baseline'))[:1500])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof_diag -o trace --output-format csv -- python3 -u -c "
import json, sys, torch
sys.path.insert(0, '$GRAFT_REPO_ROOT')
import bench
print(json.dumps(bench._diag_4096(torch, 0, torch.cuda.current_stream(0), torch.device('cuda', 0))))
" > $GRAFT_REPO_ROOT/$D/prof_diag.log 2>&1 || { echo "PROF FAILED"; tail -30 $GRAFT_REPO_ROOT/$D/prof_diag.log; exit 1; }
cd $GRAFT_REPO_ROOT
grep -E "wcoop|generic3" $D/prof_diag/trace_kernel_stats.csv | cut -d, -f1-5
echo DONE
