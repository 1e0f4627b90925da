#!/bin/bash
# round 3: the new GPU tests first, then smoke, the whole GPU suite, the default
# bench line (multi-GPU leg forced on one GPU) and the config-3 line
set -o pipefail
export TMPDIR=/tmp
P=${P:-r03d}
mkdir -p gpurun_out/$P
timeout -k 10 600 python -u -m pytest tests/test_vvc_round.py tests/test_gpu_wblk.py tests/test_areas.py tests/test_multi.py -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/$P/pytest_new.log 2>&1 || { echo "NEW TESTS FAILED"; tail -40 gpurun_out/$P/pytest_new.log; exit 1; }
grep -E "max V rel|passed|failed" gpurun_out/$P/pytest_new.log | tail -4
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$P/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/$P/smoke.log; exit 1; }
tail -3 gpurun_out/$P/smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$P/pytest_gpu.log 2>&1 || { echo "GPU SUITE FAILED"; tail -30 gpurun_out/$P/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$P/pytest_gpu.log
FPF_BENCH_MULTI=1 timeout -k 10 500 python3 -u bench.py > gpurun_out/$P/bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/$P/bench.log; exit 1; }
tail -1 gpurun_out/$P/bench.log | cut -c1-300
timeout -k 10 500 python3 -u bench.py --config 3 --steps 5 --warmup 1 > gpurun_out/$P/bench_c3.log 2>&1 || { echo "C3 FAILED"; tail -30 gpurun_out/$P/bench_c3.log; exit 1; }
tail -1 gpurun_out/$P/bench_c3.log | cut -c1-300
echo DONE
