#!/bin/bash
# Lane kernel after the spill fixes (output pointers from LDS, lazy load offsets,
# TEMP one slot ahead): its GPU tests, config 4 on the product and the ablations
# (1 no loads, 4 exactly 5 sweeps, 5 both) against the wave kernel, one SQ pass.
set -o pipefail
O=gpurun_out/r06_lane4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lane.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then echo "TESTS FAILED rc=$rc"; exit $rc; fi
for v in prod a1 a4 a5 wave; do
  unset FPF_LIB_PATH; L=1
  case $v in prod) ;; wave) L=0 ;; *) export FPF_LIB_PATH=freedm_amd/lib/abl/libfreedm_pf_lane_$v.so ;; esac
  FPF_LANE=$L timeout -k 10 200 python3 bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline --layout 0 > $O/c4_$v.json 2>&1 || { echo "C4 FAILED $v"; tail -5 $O/c4_$v.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_$v.json').readlines()[-1]); print('c4 $v', round(d['roofline']['kernel_ms'],4), 'ms', d['aggregate']['n_conv'], d['roofline']['fp64']['mean_sweeps'])"
done
unset FPF_LIB_PATH
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
FPF_LANE=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/pmc1 -o pmc1 -- python3 bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline --layout 0 > $O/pmc1.log 2>&1 || { echo "PMC FAILED"; tail -5 $O/pmc1.log; exit 1; }
echo done
