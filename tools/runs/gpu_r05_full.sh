#!/bin/bash
# Round 5: the full-output variant restructured (IL / Ib stashed, outputs after the
# sweep loop, GEN instantiations): the GPU suite, then the full-output leg against
# the previous library (freedm_amd/lib/cmp_head)
set -o pipefail
OUT=gpurun_out/r05full
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "GPU SUITE FAILED"; grep -E "FAIL|Error" $OUT/pytest_gpu.log | head -20; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for r in 1 2; do
  FPF_LIB_PATH=freedm_amd/lib/cmp_head/libfreedm_pf.so timeout -k 10 300 python3 -u tools/full_leg.py > $OUT/head_r$r.log 2>&1 || { echo "HEAD LEG FAILED"; tail -20 $OUT/head_r$r.log; exit 1; }
  tail -1 $OUT/head_r$r.log
  timeout -k 10 300 python3 -u tools/full_leg.py > $OUT/new_r$r.log 2>&1 || { echo "NEW LEG FAILED"; tail -20 $OUT/new_r$r.log; exit 1; }
  tail -1 $OUT/new_r$r.log
done
