#!/bin/bash
# GPU box: the GPU suite, the default bench line (config 2 with the CPU
# baseline) and the throughput-sized diagnostics (config 4 shard, config 3
# 2048-bus per kernel), then rocprofv3 kernel stats of configs 2 and 3.
set -o pipefail
mkdir -p gpurun_out/cfg
export TMPDIR=/tmp
O=gpurun_out/cfg
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo "BENCH C2 FAILED"; tail -30 $O/bench_c2.err; exit 1; }
tail -1 $O/bench_c2.json
timeout -k 10 300 python bench.py --config 4 --steps 20 --warmup 3 > $O/bench_c4.json 2> $O/bench_c4.err || { echo "BENCH C4 FAILED"; tail -30 $O/bench_c4.err; exit 1; }
tail -1 $O/bench_c4.json
for K in ${C3_KERNELS:-auto generic}; do
  timeout -k 10 400 python bench.py --config 3 --steps 5 --warmup 1 --kernel $K > $O/bench_c3_$K.json 2> $O/bench_c3_$K.err || { echo "BENCH C3 $K FAILED"; tail -30 $O/bench_c3_$K.err; exit 1; }
  tail -1 $O/bench_c3_$K.json
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_c2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_c2.log 2>&1 || { echo "PROF C2 FAILED"; tail -20 $GRAFT_REPO_ROOT/$O/prof_c2.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_c3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 3 --steps 5 --warmup 1 > $GRAFT_REPO_ROOT/$O/prof_c3.log 2>&1 || { echo "PROF C3 FAILED"; tail -20 $GRAFT_REPO_ROOT/$O/prof_c3.log; exit 1; }
echo DONE
