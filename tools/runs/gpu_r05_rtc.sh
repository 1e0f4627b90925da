#!/bin/bash
# Round 5: the per-plan hipRTC wave / wave-block builds compiled by the image's
# own hipRTC (fpf_rtc.cpp: rtc_api), then a same-box A/B against the static kernels.
set -o pipefail
OUT=gpurun_out/r05rtc
mkdir -p $OUT
export TMPDIR=/tmp FPF_DEBUG=1
FPF_WAVE_RTC=2048 timeout -k 10 240 python3 -u tools/wave_rtc_probe.py 123 0 > $OUT/probe_ilp_light.log 2>&1 || { echo "PROBE FAILED"; grep -v "^  File\|^    " $OUT/probe_ilp_light.log | tail -8; exit 1; }
echo "probe: $(tail -1 $OUT/probe_ilp_light.log)"
FPF_TEST_WAVE_RTC=1 timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -k specialised tests/test_gpu_wave.py tests/test_gpu_wblk.py > $OUT/pytest_rtc.log 2>&1 || { echo "PYTEST FAILED"; tail -30 $OUT/pytest_rtc.log; exit 1; }
tail -3 $OUT/pytest_rtc.log
unset FPF_DEBUG
TAG=r05rtc/ab VARIANTS="static:FPF_WAVE_RTC=0 rtc:FPF_WAVE_RTC=1" CFGS="4:1 2:1 3:1" REPS="1 2" bash tools/runs/gpu_ab_env.sh
