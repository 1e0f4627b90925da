#!/bin/bash
# round 3: the wave kernel's staged-load rows swizzled (row r at r + r/16): the
# wave-kernel GPU tests, configs 2 and 4 A/B against the same kernel without it
# (freedm_amd/lib/var_noswz), and an LDS bank-conflict pass of each
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r03v
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_wave.py tests/test_gpu_parity.py tests/test_gpu_guard.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for rep in 1 2; do
  for V in swz:- noswz:freedm_amd/lib/var_noswz/libfreedm_pf.so; do
    n=${V%%:*}; lib=${V#*:}
    ( if [ "$lib" != "-" ]; then export FPF_LIB_PATH=$lib; fi; timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline ) > $D/c24_${n}_$rep.log 2>&1 || { echo "BENCH $n FAILED"; tail -20 $D/c24_${n}_$rep.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$D/c24_${n}_$rep.log') if l.startswith('{')][-1]); print('$n c2', d['roofline']['kernel_ms'], 'c4', d['roofline_config4']['kernel_ms'])"
  done
done
for V in swz:- noswz:freedm_amd/lib/var_noswz/libfreedm_pf.so; do
  n=${V%%:*}; lib=${V#*:}
  ( cd /tmp; if [ "$lib" != "-" ]; then export FPF_LIB_PATH=$GRAFT_REPO_ROOT/$lib; fi
    timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES -d $GRAFT_REPO_ROOT/gpurun_out/pmc_r03v_${n}_1 -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/pmc_$n.log 2>&1 ) || { echo "PMC $n FAILED"; tail -20 $D/pmc_$n.log; exit 1; }
  python3 tools/pmc_sq.py r03v_$n | head -8
done
echo DONE
