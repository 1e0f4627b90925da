#!/bin/bash
# Round 6, second session: config 4 (and 2) with 2-wave workgroups (four per CU)
# and TEMP through the vector memory pipe, against the default 4-wave geometry
set -o pipefail
P=${P:-r06s2_wpb2}
mkdir -p gpurun_out/$P
export TMPDIR=/tmp
timeout -k 10 500 python3 -u tools/wave_ab.py "base:-" "tvm:FPF_WAVE_RTC_DEFS=FPF_WAVE_TEMP_VMEM" \
  "wpb2:FPF_WAVE_WPB=2+FPF_WAVE_RTC_DEFS=FPF_WAVE_TEMP_VMEM" --configs 4,2 --reps 3 > gpurun_out/$P/ab.log 2>&1 || { echo "AB FAILED"; tail -20 gpurun_out/$P/ab.log; exit 1; }
tail -4 gpurun_out/$P/ab.log
echo DONE
