#!/bin/bash
# generic-kernel parity (exact, bit-identical) incl. the full-size config-3 test,
# then config 3 current vs the previous library
set -o pipefail
mkdir -p gpurun_out/c3ab3
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vvc.py tests/test_vvc_round.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c3ab3/pytest.log 2>&1 || { tail -30 gpurun_out/c3ab3/pytest.log; exit 1; }
tail -2 gpurun_out/c3ab3/pytest.log
for rep in 1 2; do
for V in cur:- prev:FPF_LIB_PATH=$PWD/freedm_amd/lib/abl/libfreedm_pf_prev.so; do
  name=${V%%:*}; envs=${V#*:}; [ "$envs" = "-" ] && envs=""
  env $envs timeout -k 10 400 python3 -u bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c3ab3/${name}_$rep.log 2>&1 || { echo "FAILED $name"; tail -5 gpurun_out/c3ab3/${name}_$rep.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/c3ab3/${name}_$rep.log').read().strip().splitlines()[-1]); a=d['aggregate']; print('$name', 'c3 kernel %.2f ms frac %.3f loss %.10e vmin %.15f conv %d' % (d['roofline']['kernel_ms'], d['roofline']['frac'], a['loss_sum_kw'], a['vmin'], a['n_conv']))"
done; done
