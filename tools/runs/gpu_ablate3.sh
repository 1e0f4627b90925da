#!/bin/bash
# Kernel ms per launch (bench.py HIP events, config 2) for each compile-time
# ablation library in freedm_amd/lib/abl/ (tools/build_ablations.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in "$@"; do
  FPF_LIB_PATH=$PWD/freedm_amd/lib/abl/libfreedm_pf_$m.so timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/abl3_$m.log 2>&1 || { echo "ABL $m FAILED"; tail -5 gpurun_out/abl3_$m.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/abl3_$m.log').read().strip().splitlines()[-1]); print('abl $m c2 kernel_ms %.4f c4 kernel_ms %.4f' % (d['roofline']['kernel_ms'], d.get('roofline_config4', {}).get('kernel_ms', 0)))"
done
