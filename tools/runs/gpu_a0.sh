#!/bin/bash
# A0 MFMA experiment: timings, kernel trace, MFMA-busy counters.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/a0
timeout -k 10 60 $R/tools/ubench/mfma_a0 0 > $R/gpurun_out/a0/run.json 2>&1 || exit 1
cat $R/gpurun_out/a0/run.json
timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/a0/counters.txt 2>&1 || true
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/a0/trace -o run -- $R/tools/ubench/mfma_a0 0 > $R/gpurun_out/a0/trace.log 2>&1 || exit 1
for w in 1 2; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/a0/pmc$w -o run -- $R/tools/ubench/mfma_a0 $w > $R/gpurun_out/a0/pmc$w.log 2>&1 || { echo "pmc $w failed"; tail -5 $R/gpurun_out/a0/pmc$w.log; }
done
find $R/gpurun_out/a0 -name "*.csv" | head
