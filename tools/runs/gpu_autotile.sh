#!/bin/bash
# GPU box: tiled (interpreted) vs generic kernel on mid-size synthetic feeders,
# 65536 scenarios, to calibrate the auto choice (AUTO_MIN_TILE in fpf_api.cpp).
set -o pipefail
O=gpurun_out/autotile
mkdir -p $O
for N in ${SIZES:-300 512 1024}; do
  for K in tiled generic; do
    timeout -k 10 200 python bench.py --config 3 --nodes $N --scenarios ${SCEN:-0} --steps 3 --warmup 1 --kernel $K --no-specialize > $O/b_${N}_$K.json 2> $O/b_${N}_$K.err || { rc=$?; echo "BENCH $N $K FAILED rc=$rc"; tail -5 $O/b_${N}_$K.err; [ $rc -eq 1 ] && continue; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${N}_$K.json').read().strip().splitlines()[-1]); c=d['config']; print($N, c['kernel'], 'tile', c['tile'], 'kern ms %.3f' % d['roofline']['kernel_ms'], 'sweeps %.2f' % d['roofline']['fp64']['mean_sweeps'])"
  done
done
echo DONE
