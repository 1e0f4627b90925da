#!/bin/bash
# Wave-kernel ablations (diagnostic library, FPF_WAVE_DBG bits; results are wrong by design)
# then config-4 line.  Each run: kernel ms per launch from bench.py's HIP events.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export FPF_LIB_PATH=$PWD/freedm_amd/lib/libfreedm_pf_ablate.so
for spec in base:16 temp:17 sld:18 tempsld:19 nostore:112 noblk:24 nostage:272 novout:1040 noio:1296 nostore_noio:1392 empty:4096 stageonly:8192; do
  IFS=: read tag dbg <<< "$spec"
  FPF_WAVE_DBG=$dbg timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/abl_$tag.log 2>&1 || { echo "ABL $tag FAILED"; tail -5 gpurun_out/abl_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/abl_$tag.log').read().strip().splitlines()[-1]); print('$tag dbg $dbg kernel_ms %.4f' % d['roofline']['kernel_ms'])"
done
