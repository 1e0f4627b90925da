#!/bin/bash
# round 3: the wave-block kernel's segmented forward scan: its tests (the restart
# below a zeroed phase now on it), the guard tests, smoke, then config 3 A/B
# against the unsegmented kernel (freedm_amd/lib/var_unseg)
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r03m
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_wblk.py tests/test_gpu_guard.py tests/test_gpu_wcoop.py tests/test_areas.py -m gpu -x -v --timeout 200 --timeout-method thread > $D/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -60 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
grep -E "max V rel err" $D/pytest.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $D/smoke.log; exit 1; }
tail -3 $D/smoke.log
for rep in 1 2; do
  for V in seg:- unseg:freedm_amd/lib/var_unseg/libfreedm_pf.so; do
    n=${V%%:*}; lib=${V#*:}
    ( if [ "$lib" != "-" ]; then export FPF_LIB_PATH=$lib; fi; timeout -k 10 300 python3 -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline ) > $D/c3_${n}_$rep.log 2>&1 || { echo "C3 $n FAILED"; tail -20 $D/c3_${n}_$rep.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$D/c3_${n}_$rep.log') if l.startswith('{')][-1]); print('$n c3', d['roofline']['kernel_ms'])"
  done
done
echo DONE
