#!/bin/bash
# Stage split (stamps build) of the specialised kernel for several knob sets:
# STAMPS="ENV=VAL+ENV2=VAL2 ..."
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for ITEM in ${STAMPS:-DEFAULT=1}; do
  ENVS=$(echo "$ITEM" | tr '+' ' ')
  env $ENVS SPEC=1 timeout -k 10 200 python tools/stamps.py > gpurun_out/stamps_sweep.log 2>&1 || { echo "STAMPS FAILED $ITEM"; tail -20 gpurun_out/stamps_sweep.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/stamps_sweep.log') if l.startswith('{')][-1]); print('$ITEM', {k: int(v) for k, v in d['mean_cycles'].items()})"
done
