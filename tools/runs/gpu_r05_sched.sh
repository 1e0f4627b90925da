#!/bin/bash
# Round 5: the per-plan builds' machine scheduler (ILP-first vs the default)
set -o pipefail
TAG=r05sched/ab VARIANTS="base:FPF_NONE=0 wave_dflt:FPF_WAVE_RTC_SCHED=0 wblk_dflt:FPF_WBLK_RTC_SCHED=0" CFGS="2:1 4:1 3:1" REPS="1 2" bash tools/runs/gpu_ab_env.sh
