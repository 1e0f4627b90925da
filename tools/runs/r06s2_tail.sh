#!/bin/bash
# Round 6, second session: with the start marker outside the timed region, the
# round robin ending on the main stream (FPF_BENCH_RR_TAIL=1, a switch reverted
# after this run) against i % S
set -o pipefail
P=${P:-r06s2_tail}
mkdir -p gpurun_out/$P
export TMPDIR=/tmp
for r in 1 2 3 4; do
  for v in rr tail; do
    E=0; [ $v = tail ] && E=1
    FPF_BENCH_RR_TAIL=$E timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-c4 > gpurun_out/$P/${v}_$r.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/$P/${v}_$r.log; exit 1; }
    echo "$v $r $(grep -o '"value": [0-9.]*' gpurun_out/$P/${v}_$r.log | head -1)"
  done
done
echo DONE
