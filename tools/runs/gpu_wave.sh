#!/bin/bash
# Wave-kernel iteration: parity tests of the fast-mode kernels, then a short bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "wave or auto or fast_mode" > gpurun_out/wave_t.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/wave_t.log; exit 1; }
tail -1 gpurun_out/wave_t.log
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/wave_b.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/wave_b.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/wave_b.log').read().strip().splitlines()[-1]); print('value %.3e  ms/step %.4f  kernel_ms %.4f  frac %.3f' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac']))"
for G in ${GEOMS}; do
  FPF_WAVE_GEOM=$G timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/wave_b_$G.log 2>&1 || { echo "BENCH $G FAILED"; tail -20 gpurun_out/wave_b_$G.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/wave_b_$G.log').read().strip().splitlines()[-1]); print('geom $G value %.3e  ms/step %.4f  kernel_ms %.4f  frac %.3f' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac']))"
done
