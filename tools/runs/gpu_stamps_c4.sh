#!/bin/bash
# Wave-kernel stage split (stamps build) for config 2 and config 4 (first round
# and steady state: BASE = first recorded global wave).
set -o pipefail
mkdir -p gpurun_out/stamps
export TMPDIR=/tmp
run() { timeout -k 10 240 python -u tools/wave_stamps.py > gpurun_out/stamps/$1.log 2>&1 || { echo "STAMPS $1 FAILED"; tail -20 gpurun_out/stamps/$1.log; exit 1; }; echo "$1: $(tail -1 gpurun_out/stamps/$1.log)"; }
NN=123 B=4096 LAYOUT=0 run c2_l0
NN=123 B=4096 LAYOUT=1 run c2_l1
NN=123 B=131072 LAYOUT=1 MODEL=hosting BASE=0 run c4_first
NN=123 B=131072 LAYOUT=1 MODEL=hosting BASE=32768 run c4_mid
NN=123 B=131072 LAYOUT=1 MODEL=hosting BASE=32800 run c4_mid2
