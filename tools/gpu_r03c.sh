#!/bin/bash
# round 3: the batched gradient tests, the default bench (config-5 leg with the
# device-side stop, the in-process multi-GPU leg forced on one GPU), then the
# config-3 regression profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03c
timeout -k 10 600 python -u -m pytest tests/test_vvc_round.py tests/test_areas.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03c/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/r03c/pytest.log; exit 1; }
tail -2 gpurun_out/r03c/pytest.log
FPF_BENCH_MULTI=1 timeout -k 10 600 python3 -u bench.py --cpu-seconds 3 > gpurun_out/r03c/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/r03c/bench.log; exit 1; }
tail -1 gpurun_out/r03c/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
for k in ('value','ms_per_step','config5_areas','multi_gpu_inproc','config1_vvc_round'): print(k, json.dumps(d.get(k))[:600])
print('c4', d['roofline_config4']['kernel_ms'], 'c2', d['roofline']['kernel_ms'])"
bash tools/gpu_c3_regress.sh
