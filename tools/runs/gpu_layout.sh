#!/bin/bash
# GPU box: layout tests, then config 3 and config 2 (+ its config-4 leg) in both
# batch layouts; kernel ms per launch.
set -o pipefail
O=${O:-gpurun_out/layout}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_layout.py tests/test_gpu_wblk.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
show() { python3 -c "
import json
d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); r=d['roofline']; r4=d.get('roofline_config4',{})
print('%-8s %s kernel %.4f ms frac %.3f | c4 %.4f ms frac %.3f | %.1f M scen/s' % ('$2', d['config']['layout'][:10], r['kernel_ms'], r['frac'], r4.get('kernel_ms',0), r4.get('frac',0), d['value']/1e6))"; }
for L in ${LAYOUTS:-0 1}; do
  timeout -k 10 300 python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline --layout $L > $O/c3_$L.json 2> $O/c3_$L.err || { echo "C3 FAILED $L"; tail -5 $O/c3_$L.err; exit 1; }
  show $O/c3_$L.json c3
  timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --layout $L > $O/c2_$L.json 2> $O/c2_$L.err || { echo "C2 FAILED $L"; tail -5 $O/c2_$L.err; exit 1; }
  show $O/c2_$L.json c2
done
