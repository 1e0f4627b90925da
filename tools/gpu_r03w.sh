#!/bin/bash
# round 3: the wave-block kernel's Sld rows swizzled: its tests, config 3 A/B
# against the unswizzled kernel (freedm_amd/lib/var_wbold)
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r03w
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_wblk.py tests/test_areas.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for rep in 1 2; do
  for V in swz:- old:freedm_amd/lib/var_wbold/libfreedm_pf.so; do
    n=${V%%:*}; lib=${V#*:}
    ( if [ "$lib" != "-" ]; then export FPF_LIB_PATH=$lib; fi; timeout -k 10 300 python3 -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline ) > $D/c3_${n}_$rep.log 2>&1 || { echo "C3 $n FAILED"; tail -20 $D/c3_${n}_$rep.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$D/c3_${n}_$rep.log') if l.startswith('{')][-1]); print('$n c3', d['roofline']['kernel_ms'])"
  done
done
echo DONE
