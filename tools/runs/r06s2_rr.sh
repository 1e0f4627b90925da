#!/bin/bash
# Round 6, second session: the driver's command with the stream round robin
# ending on the main stream (default) against the plain i % S order
# (--rr-from-main), alternating, four pairs.
set -o pipefail
P=${P:-r06s2_rr}
mkdir -p gpurun_out/$P
export TMPDIR=/tmp
for r in 1 2 3 4; do
  for v in tail rr; do
    A=""; [ $v = rr ] && A="--rr-from-main"
    FPF_BENCH_TRACE=1 timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-c4 $A > gpurun_out/$P/${v}_$r.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/$P/${v}_$r.log; exit 1; }
    echo "$v $r $(grep -o '"value": [0-9.]*' gpurun_out/$P/${v}_$r.log | head -1)"
  done
done
echo DONE
