#!/bin/bash
# round 3 A/B: wave-kernel variants (configs 2 and 4) and the wave-block kernel
# against the round-2 tree (config 3), each twice, alternating
set -o pipefail
export TMPDIR=/tmp
NO_C3=1 VARIANTS="base:.:- ibo:.:freedm_amd/lib/var_ibo/libfreedm_pf.so ibopref:.:freedm_amd/lib/var_ibopref/libfreedm_pf.so pref:.:freedm_amd/lib/var_pref/libfreedm_pf.so" bash tools/gpu_ab_trees.sh || exit 1
mkdir -p gpurun_out/abc3
for rep in 1 2; do
  for V in old new; do
    d=.; [ $V = old ] && d=_ab/old
    ( cd $d && timeout -k 10 300 python3 -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline ) > gpurun_out/abc3/${V}_$rep.log 2>&1 || { echo "C3 $V FAILED"; tail -5 gpurun_out/abc3/${V}_$rep.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/abc3/${V}_$rep.log') if l.startswith('{')][-1]); print('$V c3', d['roofline']['kernel_ms'])"
  done
done
