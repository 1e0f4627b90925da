#!/bin/bash
# Round 6, second session: health check of HEAD (smoke, GPU suite, the driver's
# K = 20 command with the timed-region host trace) and a kernel + copy timeline
# of the K = 20 config-2 command, to split the timed region's fixed cost.
set -o pipefail
P=${P:-r06s2}
mkdir -p gpurun_out/$P
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$P/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/$P/smoke.log; exit 1; }
tail -1 gpurun_out/$P/smoke.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/$P/pytest_gpu.log 2>&1 || { echo "GPU SUITE FAILED"; tail -30 gpurun_out/$P/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$P/pytest_gpu.log
for i in 1 2; do
  FPF_BENCH_TRACE=1 timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$P/bench_k20_$i.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/$P/bench_k20_$i.log; exit 1; }
  tail -1 gpurun_out/$P/bench_k20_$i.log | cut -c1-200
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/$P/tl -o tl --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c4 > gpurun_out/$P/tl_bench.log 2>&1 || { echo "TIMELINE FAILED"; tail -30 gpurun_out/$P/tl_bench.log; exit 1; }
echo DONE
