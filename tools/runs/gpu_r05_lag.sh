#!/bin/bash
# Round 5: the sequential-order plan (tests/test_gpu_lag.py) and the wave kernels' suites
set -o pipefail
OUT=gpurun_out/r05lag
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_lag.py tests/test_gpu_parity.py tests/test_gpu_wave.py tests/test_gpu_wblk.py tests/test_gpu_layout.py tests/test_gpu_guard.py > $OUT/pytest.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAIL|Error" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
