#!/bin/bash
# Round 6, second session: the batched LU with a row permutation and the next
# pivot search fused into the update -- VVC GPU tests, then a bitwise A/B of the
# batched rounds against the previous build (its .so copied to tools/ab_lib/libfreedm_pf_oldlu.so for the run, not kept)
set -o pipefail
P=${P:-r06s2_lu}
mkdir -p gpurun_out/$P
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -k "vvc or integration" -q --timeout 200 --timeout-method thread > gpurun_out/$P/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/$P/pytest.log; exit 1; }
tail -1 gpurun_out/$P/pytest.log
for r in 1 2; do
  FPF_LIB_PATH=$PWD/tools/ab_lib/libfreedm_pf_oldlu.so timeout -k 10 200 python3 -u tools/lu_ab.py > gpurun_out/$P/old_$r.log 2>&1 || { tail -20 gpurun_out/$P/old_$r.log; exit 1; }
  timeout -k 10 200 python3 -u tools/lu_ab.py > gpurun_out/$P/new_$r.log 2>&1 || { tail -20 gpurun_out/$P/new_$r.log; exit 1; }
  echo "old $r"; grep digest gpurun_out/$P/old_$r.log; echo "new $r"; grep digest gpurun_out/$P/new_$r.log
done
echo DONE
