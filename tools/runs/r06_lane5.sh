#!/bin/bash
# Lane kernel with the finishing stores simplified (both V planes or neither):
# its GPU tests, config 4 on the product and ablation 4 (exactly 5 sweeps) against
# the wave kernel (layout 0, and its default layout 1).
set -o pipefail
O=gpurun_out/r06_lane5
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lane.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then echo "TESTS FAILED rc=$rc"; exit $rc; fi
for v in prod a4 wave; do
  unset FPF_LIB_PATH; L=1
  case $v in prod) ;; wave) L=0 ;; *) export FPF_LIB_PATH=freedm_amd/lib/abl/libfreedm_pf_lane_$v.so ;; esac
  FPF_LANE=$L timeout -k 10 200 python3 bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline --layout 0 > $O/c4_$v.json 2>&1 || { echo "C4 FAILED $v"; tail -5 $O/c4_$v.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_$v.json').readlines()[-1]); print('c4 $v', round(d['roofline']['kernel_ms'],4), 'ms', d['aggregate']['n_conv'], d['roofline']['fp64']['mean_sweeps'])"
done
unset FPF_LIB_PATH
FPF_LANE=0 timeout -k 10 200 python3 bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline --layout 1 > $O/c4_wave1.json 2>&1 || { echo "C4 FAILED wave1"; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c4_wave1.json').readlines()[-1]); print('c4 wave layout1', round(d['roofline']['kernel_ms'],4), 'ms')"
echo done
