#!/bin/bash
# Second diagnosis of the hipRTC wave build (profiles/r04rtc): the ILP-built light
# variant in a fresh process, then the default-scheduler light variant after a
# static full-output solve in the same process.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/wprobe2
export FPF_WAVE_RTC=2048 FPF_DEBUG=1
FPF_WAVE_RTC_SCHED=1 timeout -k 10 120 python3 -u tools/wave_rtc_probe.py 123 0 > gpurun_out/wprobe2/ilp_light.log 2>&1 || { echo "ILP LIGHT FAILED"; grep -v "^  File\|^    " gpurun_out/wprobe2/ilp_light.log | tail -6; exit 1; }
echo "ilp light fresh: $(tail -1 gpurun_out/wprobe2/ilp_light.log)"
FPF_WAVE_RTC_SCHED=0 timeout -k 10 120 python3 -u tools/wave_rtc_probe.py 123 0 prefull > gpurun_out/wprobe2/dflt_light_prefull.log 2>&1 || { echo "DEFAULT LIGHT AFTER FULL FAILED"; grep -v "^  File\|^    " gpurun_out/wprobe2/dflt_light_prefull.log | tail -6; exit 1; }
echo "default light after a full solve: $(tail -1 gpurun_out/wprobe2/dflt_light_prefull.log)"
echo DONE
