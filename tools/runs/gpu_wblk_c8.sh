#!/bin/bash
# Wave-block kernel geometry A/B on config 3: C = 4 (8 wavefronts) vs FPF_WBLK_C=8
# (4 wavefronts, 1 per SIMD), with the wave-block tests under C = 8 first.
set -o pipefail
O=gpurun_out/wblk_c8
mkdir -p $O
FPF_WBLK_C=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_wblk.py tests/test_gpu_layout.py -x -q --timeout 200 --timeout-method thread > $O/pytest_c8.log 2>&1 || { echo "C8 TESTS FAILED"; tail -30 $O/pytest_c8.log; exit 1; }
tail -1 $O/pytest_c8.log
for rep in 1 2; do
for C in 4 8; do
  FPF_WBLK_C=$C timeout -k 10 200 python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > $O/c3_C${C}_$rep.json 2>&1 || { echo "C3 FAILED C=$C"; tail -5 $O/c3_C${C}_$rep.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_C${C}_$rep.json').readlines()[-1]); print('C=$C', d['roofline']['kernel_ms'], d['aggregate']['n_conv'])"
done
done
