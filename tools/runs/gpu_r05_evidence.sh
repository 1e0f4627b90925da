#!/bin/bash
# Round-5 evidence, part $PART: 1 = smoke, the GPU suite, the default bench line and
# config 3; 2 = rocprofv3 stats + FETCH/WRITE passes for configs 2, 4 and 3; 3 = the
# SQ passes for configs 2, 4 and 3.  Everything under gpurun_out/$P.
set -o pipefail
P=${P:-r05}
mkdir -p gpurun_out/$P
export TMPDIR=/tmp
case ${PART:-1} in
1)
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$P/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/$P/smoke.log; exit 1; }
  tail -2 gpurun_out/$P/smoke.log
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/$P/pytest_gpu.log 2>&1 || { echo "GPU SUITE FAILED"; tail -30 gpurun_out/$P/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/$P/pytest_gpu.log
  timeout -k 10 500 python3 -u bench.py > gpurun_out/$P/bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/$P/bench.log; exit 1; }
  tail -1 gpurun_out/$P/bench.log | cut -c1-300
  timeout -k 10 500 python3 -u bench.py --config 3 --steps 5 --warmup 1 > gpurun_out/$P/bench_c3.log 2>&1 || { echo "C3 FAILED"; tail -30 gpurun_out/$P/bench_c3.log; exit 1; }
  tail -1 gpurun_out/$P/bench_c3.log | cut -c1-300
  ;;
2)
  # one stream: rocprof's per-launch average is then the bench's roofline.kernel_ms
  # (two streams overlap consecutive launches, each then lasting longer)
  for W in ${WHICH:-c2 c4 c3}; do
    case $W in
      c2) TAG=${P}_c2 ARGS="--steps 30 --warmup 5 --no-cpu-baseline --no-c4 --streams 1" bash tools/runs/gpu_profile.sh || exit 1 ;;
      c2s2) TAG=${P}_c2s2 ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-c4" bash tools/runs/gpu_profile.sh || exit 1 ;;
      c4) TAG=${P}_c4 ARGS="--config 4 --steps 10 --warmup 2 --no-cpu-baseline --streams 1" PARGS="--config 4 --steps 5 --warmup 1 --no-cpu-baseline --streams 1" bash tools/runs/gpu_profile.sh || exit 1 ;;
      c3) TAG=${P}_c3 ARGS="--config 3 --steps 5 --warmup 1 --no-cpu-baseline --streams 1" PARGS="--config 3 --steps 3 --warmup 1 --no-cpu-baseline --streams 1" bash tools/runs/gpu_profile.sh || exit 1 ;;
    esac
  done
  ;;
3)
  TAG=${P}_c2 ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-c4 --streams 1" bash tools/runs/gpu_pmc_sq.sh || exit 1
  TAG=${P}_c4 ARGS="--config 4 --steps 3 --warmup 1 --no-cpu-baseline --streams 1" bash tools/runs/gpu_pmc_sq.sh || exit 1
  TAG=${P}_c3 ARGS="--config 3 --steps 2 --warmup 1 --no-cpu-baseline --streams 1" bash tools/runs/gpu_pmc_sq.sh || exit 1
  ;;
esac
echo DONE
