#!/bin/bash
# rocprofv3 kernel trace + stats of the bench, then separate PMC passes for the
# HBM traffic of the DPF kernel (FETCH_SIZE and WRITE_SIZE need separate passes).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
ARGS=${ARGS:-"--steps 30 --warmup 5 --no-cpu-baseline --no-c4"}
# the PMC passes run the same workload as the trace, with fewer steps
PARGS=${PARGS:-"$ARGS --steps 10 --warmup 2"}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o trace --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_bench.log 2>&1 || { echo "TRACE FAILED"; tail -30 gpurun_out/prof_${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/prof_${TAG}_bench.log
ls gpurun_out/prof_$TAG
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C -d gpurun_out/pmc_${TAG}_$C -o pmc --output-format csv -- python3 bench.py $PARGS > gpurun_out/pmc_${TAG}_$C.log 2>&1 || { echo "PMC $C FAILED"; tail -30 gpurun_out/pmc_${TAG}_$C.log; exit 1; }
done
ls gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE
