#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run each) over a short bench of the
# default kernel: instruction mix, wave cycles and stall counters.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-sq}
ARGS=${ARGS:-"--steps 5 --warmup 1 --no-cpu-baseline"}
i=0
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY" ${EXTRA_SETS}; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $SET -d gpurun_out/pmc_${TAG}_$i -o pmc --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "PMC pass $i FAILED"; tail -20 gpurun_out/pmc_${TAG}_$i.log; exit 1; }
done
python3 tools/pmc_sq.py $TAG
