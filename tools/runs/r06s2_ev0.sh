#!/bin/bash
# Round 6, second session: the start event and the side streams' waits on it
# recorded before the timed region (FPF_BENCH_EV0_OUT=1) or inside it (default),
# the driver's command, alternating, four pairs
set -o pipefail
P=${P:-r06s2_ev0}
mkdir -p gpurun_out/$P
export TMPDIR=/tmp
for r in 1 2 3 4; do
  for v in in out nowait; do
    E=0; [ $v = out ] && E=1; [ $v = nowait ] && E=2
    FPF_BENCH_EV0_OUT=$E FPF_BENCH_TRACE=1 timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-c4 > gpurun_out/$P/${v}_$r.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/$P/${v}_$r.log; exit 1; }
    echo "$v $r $(grep -o '"value": [0-9.]*' gpurun_out/$P/${v}_$r.log | head -1)"
  done
done
echo DONE
