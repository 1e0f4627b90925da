#!/bin/bash
# Persistent wave-block kernel: its tests, then config 3 in both layouts against
# the previous (one workgroup per scenario) library, alternating, twice.
set -o pipefail
O=gpurun_out/persist
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_wblk.py tests/test_gpu_layout.py tests/test_multi.py tests/test_areas.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for V in new old; do
for L in 1 0; do
  if [ $V = old ]; then export FPF_LIB_PATH=freedm_amd/lib/abl/libfreedm_pf_oldwblk.so; else unset FPF_LIB_PATH; fi
  timeout -k 10 200 python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline --layout $L > $O/c3_${V}_L${L}_$rep.json 2>&1 || { echo "C3 FAILED $V $L"; tail -5 $O/c3_${V}_L${L}_$rep.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_${V}_L${L}_$rep.json').readlines()[-1]); print('$V layout $L', round(d['roofline']['kernel_ms'],3), d['aggregate']['n_conv'], d['aggregate']['loss_sum_kw'])"
done
done
done
