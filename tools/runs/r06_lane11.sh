#!/bin/bash
# Lane kernel stamps at equal work (exactly 5 sweeps) with and without the loads
# (ABL 4 / ABL 5): is the load-current phase's time the loads'?
set -o pipefail
O=gpurun_out/r06_lane11
mkdir -p $O
for v in stampsa4 stampsa1; do
  FPF_LIB_PATH=freedm_amd/lib/abl/libfreedm_pf_lane_$v.so FPF_LANE=1 timeout -k 10 300 python3 tools/lane_stamps.py > $O/$v.json 2> $O/$v.err || { echo "STAMPS FAILED $v"; tail -5 $O/$v.err; exit 1; }
  echo $v; cat $O/$v.json
done
echo done
