#!/bin/bash
# Diagnose the hipRTC wave build on the box, one launch at a time; stops at the
# first failure.  FPF_WAVE_RTC_SCHED=0 first (the default scheduler), then ILP.
set -o pipefail
mkdir -p gpurun_out/wprobe
export FPF_WAVE_RTC=2048 FPF_DEBUG=1
for s in 0 1; do
  for full in 0 1; do
    FPF_WAVE_RTC_SCHED=$s timeout -k 10 120 python3 -u tools/wave_rtc_probe.py 123 $full > gpurun_out/wprobe/p_${s}_$full.log 2>&1 || { echo "PROBE sched=$s full=$full FAILED rc=$?"; grep -v "^  File\|^    " gpurun_out/wprobe/p_${s}_$full.log | tail -12; exit 1; }
    echo "sched=$s full=$full: $(tail -1 gpurun_out/wprobe/p_${s}_$full.log)"
  done
done
echo DONE
