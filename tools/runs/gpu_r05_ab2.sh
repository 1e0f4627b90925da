#!/bin/bash
# Round 5: fresh stamps of the wave kernel (configs 2 and 4, the static build)
# and a same-box A/B of the SIMD-partner variants (stagger, static priority).
set -o pipefail
OUT=gpurun_out/r05ab2
mkdir -p $OUT
export TMPDIR=/tmp
NN=123 B=4096 LAYOUT=1 timeout -k 10 180 python3 -u tools/wave_stamps.py > $OUT/stamps_c2.log 2>&1 || { echo "STAMPS C2 FAILED"; tail -20 $OUT/stamps_c2.log; exit 1; }
echo "c2: $(tail -1 $OUT/stamps_c2.log)"
NN=123 B=131072 LAYOUT=1 MODEL=hosting BASE=16384 timeout -k 10 180 python3 -u tools/wave_stamps.py > $OUT/stamps_c4.log 2>&1 || { echo "STAMPS C4 FAILED"; tail -20 $OUT/stamps_c4.log; exit 1; }
echo "c4: $(tail -1 $OUT/stamps_c4.log)"
V=freedm_amd/lib
TAG=r05ab2/ab VARIANTS="base:FPF_WAVE_RTC=0 stag48:FPF_WAVE_RTC=0,FPF_LIB_PATH=$V/var_stag48/libfreedm_pf.so stag96:FPF_WAVE_RTC=0,FPF_LIB_PATH=$V/var_stag96/libfreedm_pf.so prio1:FPF_WAVE_RTC=0,FPF_LIB_PATH=$V/var_prio1/libfreedm_pf.so" CFGS="2:1 4:1" REPS="1 2" bash tools/runs/gpu_ab_env.sh
