#!/bin/bash
# Ablation timings of the wave kernel: FPF_WAVE_DBG bit sets (16 = exactly 5 sweeps).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag dbg extra-args
  FPF_LIB_PATH=${LIBP:-freedm_amd/lib/libfreedm_pf_ablate.so} FPF_WAVE_DBG=$2 timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline $3 > gpurun_out/${TAG:-abl}_$1.log 2>&1 || { echo "ABL $1 FAILED"; tail -5 gpurun_out/${TAG:-abl}_$1.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/${TAG:-abl}_$1.log').read().strip().splitlines()[-1]); print('$1 dbg $2 $3 kernel_ms %.4f' % d['roofline']['kernel_ms'])"
}
for spec in ${RUNS}; do
  IFS=: read tag dbg extra <<< "$spec"
  run $tag $dbg "${extra//+/ }"
done
