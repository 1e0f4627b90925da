#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/c3ab2
for rep in 1 2; do
for V in cur:- itilp:FPF_LIB_PATH=$PWD/freedm_amd/lib/abl/libfreedm_pf_gen_iterative-ilp.so; do
  name=${V%%:*}; envs=${V#*:}; [ "$envs" = "-" ] && envs=""
  env $envs timeout -k 10 400 python3 -u bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c3ab2/${name}_$rep.log 2>&1 || { echo "FAILED $name"; tail -5 gpurun_out/c3ab2/${name}_$rep.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/c3ab2/${name}_$rep.log').read().strip().splitlines()[-1]); print('$name', 'c3 kernel %.2f ms frac %.3f' % (d['roofline']['kernel_ms'], d['roofline']['frac']))"
done; done
