#!/bin/bash
# config-3 wave-block kernel: round-2 tree vs this tree vs this tree without the guard's code, rocprofv3 kernel stats
set -o pipefail
export TMPDIR=/tmp
ROOT=$(pwd)
mkdir -p gpurun_out/c3reg
run() {  # name dir lib
  ( cd $2 && if [ "$3" != "-" ]; then export FPF_LIB_PATH=$3; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/c3reg/$1 -o run -- python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > $ROOT/gpurun_out/c3reg/$1.log 2>&1 ) || { echo "FAILED $1"; tail -5 gpurun_out/c3reg/$1.log; exit 1; }
  f=$(find gpurun_out/c3reg/$1 -name "*kernel_stats.csv" | head -1)
  echo "$1: $(grep wblk $f | cut -d, -f2-4 | tail -1)"
}
for rep in 1 2; do
run old_$rep _ab/old - || exit 1
run new_$rep . - || exit 1
run ng_$rep . freedm_amd/lib/abl_ng/libfreedm_pf.so || exit 1
done
