#!/bin/bash
# Machine-scheduler A/B: the wave-block kernel (config 3) and the wave kernel
# (configs 2 and 4) built with other -amdgpu-sched-strategy settings.
set -o pipefail
A=freedm_amd/lib/abl
O=gpurun_out/sched
mkdir -p $O
for rep in 1 2; do
for V in default iterative-ilp max-ilp iterative-minreg; do
  if [ $V = default ]; then unset FPF_LIB_PATH; else export FPF_LIB_PATH=$A/libfreedm_pf_$V.so; fi
  timeout -k 10 200 python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > $O/c3_${V}_$rep.json 2>&1 || { echo "FAILED $V"; tail -3 $O/c3_${V}_$rep.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_${V}_$rep.json').readlines()[-1]); print('c3 %-18s' % '$V', round(d['roofline']['kernel_ms'], 3), d['aggregate']['n_conv'])"
done
done
unset FPF_LIB_PATH
VARIANTS="wave_default:- wave_maxilp:FPF_LIB_PATH=$A/libfreedm_pf_wave_maxilp.so" bash tools/runs/gpu_ab.sh
