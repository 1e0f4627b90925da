#!/bin/bash
# Config 3 (2048-bus x 65536, generic kernel): parity tests, then the bench
# line for the three-lane kernel and the one-lane kernel.
set -o pipefail
mkdir -p gpurun_out/c3ab
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c3ab/pytest.log 2>&1 || { tail -30 gpurun_out/c3ab/pytest.log; exit 1; }
  tail -2 gpurun_out/c3ab/pytest.log
fi
for V in three:- one:FPF_GENERIC_ONE_LANE=1; do
  name=${V%%:*}; envs=${V#*:}; [ "$envs" = "-" ] && envs=""
  env $envs timeout -k 10 400 python3 -u bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c3ab/$name.log 2>&1 || { echo "FAILED $name"; tail -5 gpurun_out/c3ab/$name.log; exit 1; }
  python3 - gpurun_out/c3ab/$name.log $name <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print("%-6s c3 kernel %.2f ms frac %.3f conv %d loss %.10e vmin %.12f" % (sys.argv[2], r["kernel_ms"], r["frac"], d["aggregate"]["n_conv"], d["aggregate"]["loss_sum_kw"], d["aggregate"]["vmin"]))
PY
done
