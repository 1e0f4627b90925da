#!/bin/bash
# Lane kernel with the loads through an LDS-DMA ring (three slots ahead): its GPU
# tests, the stamps with and without the ring, config 4 with and without it, and
# the wave kernel's config-4 layout for the box.
set -o pipefail
O=gpurun_out/r06_lane8
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lane.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then echo "TESTS FAILED rc=$rc"; exit $rc; fi
timeout -k 10 300 python3 tools/lane_stamps.py > $O/stamps_dma.json 2> $O/stamps_dma.err || { echo "STAMPS FAILED"; tail -5 $O/stamps_dma.err; exit 1; }
cat $O/stamps_dma.json
FPF_LANE_DMA=0 timeout -k 10 300 python3 tools/lane_stamps.py > $O/stamps_reg.json 2> $O/stamps_reg.err || { echo "STAMPS FAILED"; tail -5 $O/stamps_reg.err; exit 1; }
cat $O/stamps_reg.json
for v in dma reg wave1; do
  L=1; LAY=0; D=1
  case $v in reg) D=0 ;; wave1) L=0; LAY=1 ;; esac
  FPF_LANE_DMA=$D FPF_LANE=$L timeout -k 10 200 python3 bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline --layout $LAY > $O/c4_$v.json 2>&1 || { echo "C4 FAILED $v"; tail -5 $O/c4_$v.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_$v.json').readlines()[-1]); print('c4 $v', round(d['roofline']['kernel_ms'],4), 'ms', d['aggregate']['n_conv'])"
done
echo done
