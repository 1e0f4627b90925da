#!/bin/bash
# Round 5: the wave-block kernel at 2 slots per lane in 16-wavefront workgroups
# (FPF_WBLK_C=2: 4 wavefronts per SIMD at 126 VGPRs, per-plan build only) against
# the default C = 4 / 8 wavefronts: config-3 parity at full size, then config 3
# alternately, two rounds.
set -o pipefail
OUT=gpurun_out/r05wc2
mkdir -p $OUT
export TMPDIR=/tmp
FPF_DEBUG=1 FPF_WBLK_C=2 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread "tests/test_gpu_wblk.py::test_config3_wblk_full_size" > $OUT/eq_c2.log 2>&1 || { echo "EQ FAILED"; tail -30 $OUT/eq_c2.log; exit 1; }
echo "eq: $(tail -1 $OUT/eq_c2.log)"
for r in 1 2; do
for V in 4 2; do
  FPF_WBLK_C=$V timeout -k 10 300 python3 -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/c3_C${V}_r$r.log 2>&1 || { echo "C3 FAILED $V"; tail -5 $OUT/c3_C${V}_r$r.log; exit 1; }
  python3 -c "
import json
a=json.loads(open('$OUT/c3_C${V}_r$r.log').read().strip().splitlines()[-1])
print('C=$V r$r', 'c3 ms', round(a['roofline']['kernel_ms'],4), 'ms/step', round(a['ms_per_step'],4), 'rtc', a['config'].get('wave_rtc_builds'), 'conv', a['aggregate']['n_conv'])"
done
done
