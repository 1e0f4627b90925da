#!/bin/bash
# round 3: the wave kernel's staged loads in slot order (STG rows = slots, not Dl
# rows): the wave-kernel GPU tests, then configs 2 and 4 A/B against the
# previous kernel (freedm_amd/lib/var_old) and an LDS bank-conflict pass
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r03h
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_wave.py tests/test_gpu_parity.py tests/test_gpu_guard.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for rep in 1 2; do
  for V in new:- old:freedm_amd/lib/var_old/libfreedm_pf.so; do
    n=${V%%:*}; lib=${V#*:}
    ( if [ "$lib" != "-" ]; then export FPF_LIB_PATH=$lib; fi; timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline ) > $D/c24_${n}_$rep.log 2>&1 || { echo "BENCH $n FAILED"; tail -20 $D/c24_${n}_$rep.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$D/c24_${n}_$rep.log') if l.startswith('{')][-1]); print('$n c2', d['roofline']['kernel_ms'], 'c4', d['roofline_config4']['kernel_ms'])"
  done
done
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES -d $GRAFT_REPO_ROOT/gpurun_out/pmc_r03h_lds_1 -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/pmc_lds.log 2>&1 || { echo "PMC FAILED"; tail -20 $GRAFT_REPO_ROOT/$D/pmc_lds.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 tools/pmc_sq.py r03h_lds 2>&1 | head -20
echo DONE
