#!/bin/bash
# Round 6, second session: HSA signal waits by polling (HSA_ENABLE_INTERRUPT=0)
# against the default, the driver's command, alternating, four pairs
set -o pipefail
P=${P:-r06s2_intr}
mkdir -p gpurun_out/$P
export TMPDIR=/tmp
for r in 1 2 3 4; do
  for v in def poll; do
    if [ $v = poll ]; then
      HSA_ENABLE_INTERRUPT=0 FPF_BENCH_TRACE=1 timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-c4 > gpurun_out/$P/${v}_$r.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/$P/${v}_$r.log; exit 1; }
    else
      FPF_BENCH_TRACE=1 timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-c4 > gpurun_out/$P/${v}_$r.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/$P/${v}_$r.log; exit 1; }
    fi
    echo "$v $r $(grep -o '"value": [0-9.]*' gpurun_out/$P/${v}_$r.log | head -1)"
  done
done
echo DONE
