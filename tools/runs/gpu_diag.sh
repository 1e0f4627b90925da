#!/bin/bash
# Diagnostics on the GPU box: per-stage stamp split of the specialised kernel
# (diagnostic build) and the LDS/chain microbenchmarks.  Each step time-limited;
# the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/ubench/chain2_bin > gpurun_out/chain2.log 2>&1 || { echo "CHAIN2 FAILED"; tail gpurun_out/chain2.log; exit 1; }
cat gpurun_out/chain2.log
timeout -k 10 120 tools/ubench/chain_bin > gpurun_out/chain.log 2>&1 || { echo "CHAIN FAILED"; tail gpurun_out/chain.log; exit 1; }
cat gpurun_out/chain.log
for SPEC in 1 0; do
  SPEC=$SPEC timeout -k 10 200 python tools/stamps.py > gpurun_out/stamps_$SPEC.log 2>&1 || { echo "STAMPS FAILED"; tail -20 gpurun_out/stamps_$SPEC.log; exit 1; }
  tail -1 gpurun_out/stamps_$SPEC.log
done
