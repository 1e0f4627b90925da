#!/bin/bash
# Round 5: wave-kernel stamps by sweep index (config 2 and config-4 steady state)
set -o pipefail
OUT=gpurun_out/r05st4
mkdir -p $OUT
export TMPDIR=/tmp
NN=123 B=4096 LAYOUT=1 timeout -k 10 180 python3 -u tools/wave_stamps.py > $OUT/wave_c2.log 2>&1 || { echo "STAMPS C2 FAILED"; tail -20 $OUT/wave_c2.log; exit 1; }
tail -1 $OUT/wave_c2.log
NN=123 B=131072 LAYOUT=1 MODEL=hosting BASE=16384 timeout -k 10 180 python3 -u tools/wave_stamps.py > $OUT/wave_c4.log 2>&1 || { echo "STAMPS C4 FAILED"; tail -20 $OUT/wave_c4.log; exit 1; }
tail -1 $OUT/wave_c4.log
