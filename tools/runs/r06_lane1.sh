#!/bin/bash
# Round 6, first lane-kernel run: its GPU tests, then config 4 (131 072 hosting
# scenarios, scenario-fastest batch) on the lane kernel against the wave kernel
# (both layouts), and config 2 on each.
set -o pipefail
O=gpurun_out/r06_lane1
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_lane.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -15 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS ABORTED rc=$rc"; exit $rc; fi
for run in "lane 1 0" "wave 0 0" "wave 0 1"; do
  set -- $run
  FPF_LANE=$2 timeout -k 10 200 python3 bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline --layout $3 > $O/c4_$1_L$3.json 2>&1 || { echo "C4 FAILED $run"; tail -5 $O/c4_$1_L$3.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_$1_L$3.json').readlines()[-1]); print('c4 $run', round(d['roofline']['kernel_ms'],4), 'ms', round(d['roofline']['frac'],3), d['aggregate']['n_conv'], d['aggregate']['loss_sum_kw'], d['roofline']['fp64']['mean_sweeps'])"
done
for run in "lane 1 0" "wave 0 1"; do
  set -- $run
  FPF_LANE=$2 timeout -k 10 200 python3 bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline --no-c4 --layout $3 > $O/c2_$1_L$3.json 2>&1 || { echo "C2 FAILED $run"; tail -5 $O/c2_$1_L$3.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c2_$1_L$3.json').readlines()[-1]); print('c2 $run', round(d['value']/1e6,1), 'M/s kernel', round(d['roofline']['kernel_ms']*1e3,1), 'us')"
done
