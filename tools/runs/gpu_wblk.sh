#!/bin/bash
# GPU box: the wave-block kernel's tests, then the whole GPU suite, then the
# config-3 bench line (fast mode = the wave-block kernel) with rocprofv3 stats,
# then the default bench line.  Every GPU step has its own limit; stop at the first failure.
set -o pipefail
O=${O:-gpurun_out/wblk}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_wblk.py -x -v --timeout 200 --timeout-method thread > $O/pytest_wblk.log 2>&1 || { echo "WBLK TESTS FAILED"; tail -40 $O/pytest_wblk.log; exit 1; }
tail -8 $O/pytest_wblk.log
timeout -k 10 300 python bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { echo "BENCH C3 FAILED"; tail -30 $O/bench_c3.err; exit 1; }
tail -1 $O/bench_c3.json | cut -c1-600
R=$GRAFT_REPO_ROOT
if [ -n "$PROF" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > $R/$O/prof.log 2>&1 || { echo "PROF FAILED"; tail -20 $R/$O/prof.log; exit 1; }
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $C -d $R/$O/pmc_$C -o pmc --output-format csv -- python3 $R/bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/pmc_$C.log 2>&1 || { echo "PMC $C FAILED"; tail -20 $R/$O/pmc_$C.log; exit 1; }
  done
  cd $R
fi
if [ -n "$SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "GPU SUITE FAILED"; tail -40 $O/pytest_gpu.log; exit 1; }
  tail -3 $O/pytest_gpu.log
fi
echo DONE
