#!/bin/bash
# Round 5: stamps of the wave-block kernel (config 3) and of the wave kernel's
# 4-wave geometry at config 2 (the stamps build: static kernels).
set -o pipefail
OUT=gpurun_out/r05st3
mkdir -p $OUT
export TMPDIR=/tmp
NN=2048 B=65536 BASE=32768 timeout -k 10 240 python3 -u tools/wblk_stamps.py > $OUT/wblk_c3.log 2>&1 || { echo "WBLK STAMPS FAILED"; tail -20 $OUT/wblk_c3.log; exit 1; }
echo "c3: $(tail -1 $OUT/wblk_c3.log)"
NN=123 B=4096 LAYOUT=1 timeout -k 10 180 python3 -u tools/wave_stamps.py > $OUT/wave_c2_wpb4.log 2>&1 || { echo "STAMPS C2 FAILED"; tail -20 $OUT/wave_c2_wpb4.log; exit 1; }
echo "c2: $(tail -1 $OUT/wave_c2_wpb4.log)"
