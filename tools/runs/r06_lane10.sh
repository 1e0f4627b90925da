#!/bin/bash
# Lane kernel: every other CU's first workgroup started late (FPF_LANE_STAGGER
# cycles) so that the CUs' load-current bursts do not coincide; config 4.
set -o pipefail
O=gpurun_out/r06_lane10
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lane.py -x -q -m gpu --timeout 300 --timeout-method thread -k "oracle and 123" > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; echo "TESTS FAILED"; exit 1; }
tail -1 $O/pytest.log
for v in 0 8000 16000 24000 32000 48000 w; do
  L=1; LAY=0
  if [ $v = w ]; then L=0; LAY=1; fi
  FPF_LANE_STAGGER=$v FPF_LANE=$L timeout -k 10 200 python3 bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline --layout $LAY > $O/c4_$v.json 2>&1 || { echo "C4 FAILED $v"; tail -5 $O/c4_$v.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_$v.json').readlines()[-1]); print('c4 stagger $v', round(d['roofline']['kernel_ms'],4), 'ms', d['aggregate']['n_conv'])"
done
FPF_LANE_STAGGER=24000 FPF_LANE=1 timeout -k 10 300 python3 tools/lane_stamps.py > $O/stamps_24k.json 2> $O/stamps.err || { echo "STAMPS FAILED"; tail -5 $O/stamps.err; exit 1; }
cat $O/stamps_24k.json
echo done
