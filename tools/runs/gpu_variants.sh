#!/bin/bash
# Wave-kernel variants: parity (GPU wave + parity tests) then kernel ms for
# configs 2 and 4.  VARIANTS="tag:libpath:env ..." (env as K=V,K=V).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in $VARIANTS; do
  IFS=: read tag lib envs <<< "$spec"
  [ "$lib" = "-" ] && lib=$PWD/freedm_amd/lib/libfreedm_pf.so
  export FPF_LIB_PATH=$lib
  unset FPF_WAVE_WPB
  for kv in ${envs//,/ }; do export "$kv"; done
  if [ -n "$TESTS" ]; then
    timeout -k 10 300 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/var_${tag}_tests.txt 2>&1 || { echo "$tag TESTS FAILED"; tail -20 gpurun_out/var_${tag}_tests.txt; exit 1; }
    echo "$tag tests: $(tail -1 gpurun_out/var_${tag}_tests.txt)"
  fi
  for cfg in ${CONFIGS:-2 4}; do
    timeout -k 10 180 python bench.py --config $cfg --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline > gpurun_out/var_${tag}_c$cfg.log 2>&1 || { echo "$tag c$cfg FAILED"; tail -5 gpurun_out/var_${tag}_c$cfg.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/var_${tag}_c$cfg.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag c$cfg kernel_ms %.4f frac %.4f value %.4g tile %s' % (r['kernel_ms'], r['frac'], d['value'], d['config']['tile']))"
  done
done
