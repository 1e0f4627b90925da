#!/bin/bash
# round 3: the multi-area loop with fused exchange kernels and an adaptive first chunk
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r03o
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_areas.py tests/test_gpu_wblk.py::test_wblk_areas_equal_monolithic tests/test_gpu_wcoop.py::test_wcoop_areas_equal_monolithic -m gpu -x -v --timeout 200 --timeout-method thread > $D/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -60 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
for rep in 1 2; do timeout -k 10 200 python3 -u tools/c5_leg.py > $D/c5_$rep.log 2>&1 || { echo "C5 FAILED"; tail -20 $D/c5_$rep.log; exit 1; }; tail -1 $D/c5_$rep.log; done
echo DONE
