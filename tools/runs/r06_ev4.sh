#!/bin/bash
# Round-6: the lane kernel on config 4 (FPF_LANE=1, scenario-fastest batch) under
# rocprofv3 -- kernel trace + stats, FETCH / WRITE passes, SQ passes.
set -o pipefail
export TMPDIR=/tmp
export FPF_LANE=1
TAG=r06_c4lane ARGS="--config 4 --steps 10 --warmup 2 --no-cpu-baseline --streams 1 --layout 0" PARGS="--config 4 --steps 5 --warmup 1 --no-cpu-baseline --streams 1 --layout 0" bash tools/runs/gpu_profile.sh || exit 1
TAG=r06_c4lane ARGS="--config 4 --steps 3 --warmup 1 --no-cpu-baseline --streams 1 --layout 0" bash tools/runs/gpu_pmc_sq.sh || exit 1
echo DONE1
# config 3: the static wave-block build against the per-plan one (FPF_WAVE_RTC=0),
# SQ pass 2 only (the bank conflicts)
unset FPF_LANE
EXTRA_SETS="" TAG=r06_c3static ARGS="--config 3 --steps 2 --warmup 1 --no-cpu-baseline --streams 1" FPF_WAVE_RTC=0 bash tools/runs/gpu_pmc_sq.sh || exit 1
echo DONE2
