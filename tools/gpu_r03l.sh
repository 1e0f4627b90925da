#!/bin/bash
# round 3: paired kernel in the multi-area solve and under the convergence guard
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r03l
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_gpu_wcoop.py tests/test_gpu_guard.py -m gpu -x -v --timeout 200 --timeout-method thread > $D/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -60 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
echo DONE
