#!/bin/bash
# round-3 check: the changed GPU tests, then builds A/B (round-2 final vs this tree), then guard on/off on this tree
set -o pipefail
mkdir -p gpurun_out/r03b
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_areas.py tests/test_integration.py tests/test_gpu_layout.py tests/test_gpu_guard.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03b/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/r03b/pytest.log; exit 1; }
tail -2 gpurun_out/r03b/pytest.log
VARIANTS="old:_ab/old:- new:.:-" bash tools/gpu_ab_trees.sh || exit 1
timeout -k 10 400 python -u tools/wave_ab.py "guard:-" "noguard:AB_NO_GUARD=1" --configs 2,4,3 --reps 2 > gpurun_out/r03b/guard_ab.log 2>&1 || { echo "GUARD AB FAILED"; tail -5 gpurun_out/r03b/guard_ab.log; exit 1; }
tail -4 gpurun_out/r03b/guard_ab.log
