#!/bin/bash
# GPU box: the GPU suite, then config 3 (2048-bus x 65536) on the auto kernel:
# bench line, rocprofv3 kernel stats and HBM PMC passes (FETCH_SIZE, then WRITE_SIZE).
set -o pipefail
O=gpurun_out/c3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python bench.py --config 3 --steps 5 --warmup 1 > $O/bench_c3.json 2> $O/bench_c3.err || { echo "BENCH C3 FAILED"; tail -30 $O/bench_c3.err; exit 1; }
tail -1 $O/bench_c3.json
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --config 3 --steps 5 --warmup 1 > $R/$O/prof.log 2>&1 || { echo "PROF FAILED"; tail -20 $R/$O/prof.log; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C -d $R/$O/pmc_$C -o pmc --output-format csv -- python3 $R/bench.py --config 3 --steps 3 --warmup 1 > $R/$O/pmc_$C.log 2>&1 || { echo "PMC $C FAILED"; tail -20 $R/$O/pmc_$C.log; exit 1; }
done
echo DONE
