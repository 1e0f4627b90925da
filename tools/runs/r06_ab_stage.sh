#!/bin/bash
# Config 4: the round-5 library, the current one (idle waves' staging loads based
# on the tile) and variant vb (only the wave's own chunks loaded), alternating;
# then vb's exact-size-buffer and ragged-batch tests.
set -o pipefail
O=gpurun_out/r06_ab_stage
mkdir -p $O
for rep in 1 2 3 4; do
  for v in r05 cur vb; do
    unset FPF_LIB_PATH
    [ $v != cur ] && export FPF_LIB_PATH=freedm_amd/lib/abl/libfreedm_pf_$v.so
    timeout -k 10 200 python3 bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline > $O/c4_${v}_$rep.json 2>&1 || { echo "FAILED $v"; tail -5 $O/c4_${v}_$rep.json; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c4_${v}_$rep.json').read().strip().splitlines()[-1]); print('$v rep $rep', round(d['roofline']['kernel_ms'],4), 'ms')"
  done
done
FPF_LIB_PATH=freedm_amd/lib/abl/libfreedm_pf_vb.so timeout -k 10 300 python -u -m pytest tests/test_gpu_exact_buffers.py tests/test_gpu_wave.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_vb.log 2>&1; rc=$?; tail -2 $O/pytest_vb.log
exit $rc
