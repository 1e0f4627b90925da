#!/bin/bash
# round 3: the wave kernel's dynamic VALU mix (config 2): which SQ_INSTS_VALU_* counters exist, then passes of them
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r03t
mkdir -p $D
i=0
for SET in "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_INSTS_VALU" \
           "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_WAVES SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $SET -d gpurun_out/pmc_r03t_$i -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-c4 > $D/pmc_$i.log 2>&1 || { echo "PMC $i FAILED"; tail -5 $D/pmc_$i.log; exit 1; }
done
python3 tools/pmc_sq.py r03t | head -30
echo DONE
