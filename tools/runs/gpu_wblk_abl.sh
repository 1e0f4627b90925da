#!/bin/bash
# Wave-block kernel diagnostics on config 3: ablation libraries (tools/build_ablations.sh
# wblk 1 2 3 4) and a batch-size sweep of the product library; kernel ms per launch.
set -o pipefail
O=gpurun_out/wblk_abl
mkdir -p $O
show() { python3 -c "
import json,sys
d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); r=d['roofline']
print('%-10s B=%6d kernel %.3f ms  conv %d  sweeps %.2f' % ('$2', d['config']['scenarios_per_gpu'], r['kernel_ms'], d['aggregate']['n_conv'], r['fp64']['mean_sweeps']))"; }
for V in ${VARIANTS:-0 1 2 3 4}; do
  if [ $V = 0 ]; then LP=""; else LP=freedm_amd/lib/abl/libfreedm_pf_wblk_$V.so; fi
  FPF_LIB_PATH=$LP timeout -k 10 200 python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > $O/abl_$V.json 2> $O/abl_$V.err || { echo "FAILED $V"; tail -5 $O/abl_$V.err; exit 1; }
  show $O/abl_$V.json abl$V
done
for B in ${BS:-256 1024 4096 16384}; do
  timeout -k 10 200 python3 bench.py --config 3 --scenarios $B --steps 5 --warmup 1 --no-cpu-baseline > $O/bs_$B.json 2> $O/bs_$B.err || { echo "FAILED B=$B"; tail -5 $O/bs_$B.err; exit 1; }
  show $O/bs_$B.json bs
done
