#!/bin/bash
# round 3: the paired wave-block kernel (fpf_wcoop.hip, 2049..4096 branches):
# its GPU tests, then the wave-block tests (the shared launcher)
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r03i
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_wcoop.py -m gpu -x -v --timeout 150 --timeout-method thread > $D/pytest_wcoop.log 2>&1 || { echo "WCOOP TESTS FAILED"; tail -60 $D/pytest_wcoop.log; exit 1; }
tail -3 $D/pytest_wcoop.log
grep -E "max V rel" $D/pytest_wcoop.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_wblk.py tests/test_vvc_round.py -m gpu -x -q --timeout 150 --timeout-method thread > $D/pytest_wblk.log 2>&1 || { echo "WBLK TESTS FAILED"; tail -40 $D/pytest_wblk.log; exit 1; }
tail -1 $D/pytest_wblk.log
echo DONE
