#!/bin/bash
# One GPU-box pass: the GPU tests in $TESTS (default: the whole -m gpu suite),
# then, if they pass, the same-box A/B of $VARIANTS (tools/runs/gpu_ab_env.sh).
#   TAG=r04d TESTS="tests/test_gpu_wave.py" VARIANTS="prev:FPF_LIB_PATH=... new:FPF_X=1" bash tools/runs/gpu_tests_ab.sh
set -o pipefail
TAG=${TAG:-ab}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
if [ -n "${TESTS-x}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-800} python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:--m gpu tests} \
    > gpurun_out/$TAG/pytest.log 2>&1
  rc=$?
  tail -5 gpurun_out/$TAG/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
[ -z "$VARIANTS" ] || TAG=$TAG bash tools/runs/gpu_ab_env.sh
