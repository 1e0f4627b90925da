#!/bin/bash
# A/B on one box: the 4096-bus leg with the committed exchange (lib_exp) and the data-polled one (lib), twice each
set -o pipefail
mkdir -p gpurun_out/r03ac
for i in 1 2; do
  FPF_LIB_PATH=$PWD/freedm_amd/lib_exp/libfreedm_pf.so timeout -k 10 200 python -u tools/coop_leg.py > gpurun_out/r03ac/old$i.log 2>&1 &&
  timeout -k 10 200 python -u tools/coop_leg.py > gpurun_out/r03ac/new$i.log 2>&1 || exit 1
done
