#!/bin/bash
# Round 6, second session: config 5 with the C <= 2 geometries back on 8-wave
# workgroups (fpf_api.cpp: wave_small_wpb_regs_ok), its timeline, the area tests;
# and the per-phase priority switch on config 2 again (5 reps).
set -o pipefail
P=${P:-r06s2_c5}
mkdir -p gpurun_out/$P
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_areas.py -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/$P/pytest_areas.log 2>&1 || { echo "AREAS TESTS FAILED"; tail -20 gpurun_out/$P/pytest_areas.log; exit 1; }
tail -1 gpurun_out/$P/pytest_areas.log
TAG=$P/c5 bash tools/runs/gpu_c5.sh || exit 1
python3 tools/c5_timeline.py gpurun_out/$P/c5/kt > gpurun_out/$P/c5_timeline.txt && tail -22 gpurun_out/$P/c5_timeline.txt
timeout -k 10 300 python3 -u tools/wave_ab.py "base:-" "dp1:FPF_WAVE_RTC_DEFS=FPF_WAVE_DPRIO=1" --configs 2 --reps 5 > gpurun_out/$P/ab_c2.log 2>&1 || { echo "AB FAILED"; tail -20 gpurun_out/$P/ab_c2.log; exit 1; }
tail -3 gpurun_out/$P/ab_c2.log
echo DONE
