#!/bin/bash
# Round 6, second session: per-phase issue priority (FPF_WAVE_DPRIO, per-plan
# build) A/B on configs 2 and 4, then the config-5 timeline of today's library.
set -o pipefail
P=${P:-r06s2_dprio}
mkdir -p gpurun_out/$P
export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/wave_ab.py "base:-" "dp1:FPF_WAVE_RTC_DEFS=FPF_WAVE_DPRIO=1" \
  "dp2:FPF_WAVE_RTC_DEFS=FPF_WAVE_DPRIO=2" --configs 2,4 --reps 3 > gpurun_out/$P/ab.log 2>&1 || { echo "AB FAILED"; tail -20 gpurun_out/$P/ab.log; exit 1; }
tail -4 gpurun_out/$P/ab.log
TAG=$P/c5 bash tools/runs/gpu_c5.sh || exit 1
python3 tools/c5_timeline.py gpurun_out/$P/c5/kt > gpurun_out/$P/c5_timeline.txt && tail -25 gpurun_out/$P/c5_timeline.txt
echo DONE
