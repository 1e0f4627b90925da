#!/bin/bash
# Iteration pass on the GPU box: a subset of the GPU tests, then the bench line
# (config 2 + the config-4 roofline, no CPU baseline).  Each GPU step has its own
# time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-"tests/test_gpu_parity.py tests/test_gpu_wave.py tests/test_areas.py"}
TAG=${TAG:-iter}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
  tail -6 gpurun_out/${TAG}_pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python -u bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline $BENCH_ARGS > gpurun_out/${TAG}_bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
python3 - gpurun_out/${TAG}_bench.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r, r4 = d["roofline"], d.get("roofline_config4", {})
print("c2 kernel_ms %.4f frac %.4f | c4 kernel_ms %s frac %s | n_conv %d value %.4g" % (
    r["kernel_ms"], r["frac"], r4.get("kernel_ms"), r4.get("frac"), d["aggregate"]["n_conv"], d["value"]))
PY
