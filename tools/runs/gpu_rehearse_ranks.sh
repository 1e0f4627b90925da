#!/bin/bash
# The multi-rank bench path (barrier, max-over-ranks time, aggregate all-reduce)
# with the HIP kernels: 2 ranks sharing the box's one GPU over gloo.
set -o pipefail
mkdir -p gpurun_out
FPF_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --no-c4 --no-cpu-baseline \
  > gpurun_out/rehearse2.log 2>&1 || { echo "FAILED"; tail -30 gpurun_out/rehearse2.log; exit 1; }
grep '^{' gpurun_out/rehearse2.log | cut -c1-700
