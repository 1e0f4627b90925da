#!/bin/bash
# Compile-time ablation builds of the wave kernel (FPF_WAVE_ABL=<bits>, see the
# DBG() uses in fpf_wave.hip) or, with "wblk" as the first argument, of the
# wave-block kernel (FPF_WBLK_ABL, WABL() in fpf_wblk.hip): one library per bit
# set in freedm_amd/lib/abl/.
# Diagnostic only -- results are wrong by design.
set -e
cd "$(dirname "$0")/../freedm_amd/csrc"
OUT=../lib/abl
mkdir -p $OUT
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result -I../../include"
if [ "$1" = wblk ]; then
  shift
  OBJS="../lib/fpf_api.o ../lib/fpf_generic.o ../lib/fpf_tiled.o ../lib/fpf_rtc.o ../lib/fpf_selftest.o ../lib/fpf_wave.o ../lib/fpf_layout.o ../lib/fpf_vvc.o ../lib/fpf_multi.o ../lib/fpf_areas.o ../lib/fpf_areas_kernels.o ../lib/fpf_vvc_grad.o"
  for m in "$@"; do /opt/rocm/bin/hipcc $FLAGS -DFPF_WBLK_ABL=$m -c fpf_wblk.hip -o $OUT/wblk_$m.o & done
  wait
  for m in "$@"; do /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libfreedm_pf_wblk_$m.so $OBJS $OUT/wblk_$m.o -lhiprtc -lrccl; done
  exit 0
fi
OBJS="../lib/fpf_api.o ../lib/fpf_generic.o ../lib/fpf_tiled.o ../lib/fpf_rtc.o ../lib/fpf_selftest.o ../lib/fpf_vvc.o ../lib/fpf_multi.o ../lib/fpf_areas.o ../lib/fpf_areas_kernels.o ../lib/fpf_vvc_grad.o ../lib/fpf_wblk.o ../lib/fpf_layout.o"
for m in "$@"; do
  /opt/rocm/bin/hipcc $FLAGS -DFPF_WAVE_ABL=$m -c fpf_wave.hip -o $OUT/wave_$m.o &
done
wait
for m in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libfreedm_pf_$m.so $OBJS $OUT/wave_$m.o -lhiprtc -lrccl
done
