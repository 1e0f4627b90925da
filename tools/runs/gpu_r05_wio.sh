#!/bin/bash
# Round 5: per-wave IO in the wave kernel -- parity first, then a same-box A/B
# against the workgroup IO (FPF_WAVE_WG_IO=1), plus two register/prefetch knobs.
set -o pipefail
OUT=gpurun_out/r05wio
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_wave.py tests/test_gpu_layout.py tests/test_gpu_parity.py tests/test_gpu_guard.py > $OUT/pytest.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAIL|Error|error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
V=freedm_amd/lib
TAG=r05wio/ab VARIANTS="wgio:FPF_WAVE_WG_IO=1 wio:FPF_NONE=0 wio_wpb4:FPF_WAVE_WPB=4,FPF_WAVE_RTC=1 sldpref:FPF_WAVE_RTC=0,FPF_LIB_PATH=$V/var_sldpref/libfreedm_pf.so ibolds:FPF_WAVE_RTC=0,FPF_LIB_PATH=$V/var_ibolds/libfreedm_pf.so wgio_nortc:FPF_WAVE_WG_IO=1,FPF_WAVE_RTC=0" CFGS="2:1 4:1" REPS="1 2" bash tools/runs/gpu_ab_env.sh
