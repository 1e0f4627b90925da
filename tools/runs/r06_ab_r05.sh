#!/bin/bash
# Same-box A/B: the round-5 library (built from commit 1093310 into
# freedm_amd/lib/abl/libfreedm_pf_r05.so) against the current one, alternating,
# on the driver's command (config 2, K = 20) and config 4.
set -o pipefail
O=gpurun_out/r06_ab_r05
mkdir -p $O
for rep in ${REPS:-1 2}; do
  for v in r05 r06; do
    unset FPF_LIB_PATH
    [ $v = r05 ] && export FPF_LIB_PATH=freedm_amd/lib/abl/libfreedm_pf_r05.so
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/c2_${v}_$rep.json 2>&1 || { echo "FAILED $v"; tail -5 $O/c2_${v}_$rep.json; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c2_${v}_$rep.json').read().strip().splitlines()[-1]); print('$v rep $rep', round(d['value']/1e6,1), 'M/s', 'serial', round(d['roofline']['kernel_ms']*1e3,2), 'us', 'c4', round(d['roofline_config4']['kernel_ms'],4), 'ms')"
  done
done
echo done
