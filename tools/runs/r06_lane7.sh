#!/bin/bash
# Lane kernel: where a sweep's time goes (stamps build, tools/lane_stamps.py), the
# load currents without the per-slot scheduling barrier (sb0), the product and the
# wave kernel's config-4 layout for the box.
set -o pipefail
O=gpurun_out/r06_lane7
mkdir -p $O
timeout -k 10 300 python3 tools/lane_stamps.py > $O/stamps.json 2> $O/stamps.err || { echo "STAMPS FAILED"; tail -5 $O/stamps.err; exit 1; }
cat $O/stamps.json
for v in prod sb0 wave1; do
  unset FPF_LIB_PATH; L=1; LAY=0
  case $v in prod) ;; wave1) L=0; LAY=1 ;; *) export FPF_LIB_PATH=freedm_amd/lib/abl/libfreedm_pf_lane_$v.so ;; esac
  FPF_LANE=$L timeout -k 10 200 python3 bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline --layout $LAY > $O/c4_$v.json 2>&1 || { echo "C4 FAILED $v"; tail -5 $O/c4_$v.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_$v.json').readlines()[-1]); print('c4 $v', round(d['roofline']['kernel_ms'],4), 'ms', d['aggregate']['n_conv'])"
done
echo done
