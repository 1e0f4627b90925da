#!/bin/bash
# round 3: warm-started area solves (tests, the bench's config-5 leg), then the
# profile evidence (tools/gpu_r03e.sh), then config 3 without the guard's code
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03g
timeout -k 10 600 python -u -m pytest tests/test_areas.py tests/test_gpu_wave.py tests/test_gpu_wblk.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03g/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/r03g/pytest.log; exit 1; }
tail -1 gpurun_out/r03g/pytest.log
timeout -k 10 500 python3 -u bench.py --cpu-seconds 3 > gpurun_out/r03g/bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/r03g/bench.log; exit 1; }
tail -1 gpurun_out/r03g/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['roofline']['kernel_ms'], 'c4', d['roofline_config4']['kernel_ms'], 'c3', d['roofline_config3']['kernel_ms']); print(json.dumps(d['config5_areas']))"
P=r03g bash tools/gpu_r03e.sh || exit 1
for rep in 1 2; do
  for V in cur:- ng:freedm_amd/lib/abl_ng/libfreedm_pf.so; do
    n=${V%%:*}; lib=${V#*:}
    ( if [ "$lib" != "-" ]; then export FPF_LIB_PATH=$lib; fi; timeout -k 10 300 python3 -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline ) > gpurun_out/r03g/c3_${n}_$rep.log 2>&1 || { echo "C3 $n FAILED"; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r03g/c3_${n}_$rep.log') if l.startswith('{')][-1]); print('$n c3', d['roofline']['kernel_ms'])"
  done
done
