#!/bin/bash
# Lane kernel ablations on config 4 (FPF_LANE_ABL: 1 loads from a constant, 2 no
# LDS gathers, 3 both; results wrong by design) and its SQ counters.
set -o pipefail
O=gpurun_out/r06_lane2
mkdir -p $O
for v in prod 1 2 3; do
  if [ $v = prod ]; then unset FPF_LIB_PATH; else export FPF_LIB_PATH=freedm_amd/lib/abl/libfreedm_pf_laneabl$v.so; fi
  FPF_LANE=1 timeout -k 10 200 python3 bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline --layout 0 > $O/c4_$v.json 2>&1 || { echo "C4 FAILED $v"; tail -5 $O/c4_$v.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_$v.json').readlines()[-1]); print('c4 abl $v', round(d['roofline']['kernel_ms'],4), 'ms')"
done
unset FPF_LIB_PATH
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
FPF_LANE=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_WAVES -d $O/pmc1 -o pmc1 -- python3 bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline --layout 0 > $O/pmc1.log 2>&1 || { echo "PMC FAILED"; tail -5 $O/pmc1.log; exit 1; }
find $O/pmc1 -name "*.csv" | head
