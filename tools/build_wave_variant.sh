#!/bin/bash
# freedm_amd/lib/var_<name>/libfreedm_pf.so: the product library with fpf_wave.hip
# built with extra -D flags (experiments; load with FPF_LIB_PATH)
set -e
name=$1; shift
cd "$(dirname "$0")/../freedm_amd/csrc"
make -s -j8 >/dev/null
out=../lib/var_$name
mkdir -p $out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result -I../../include \
  -mllvm -amdgpu-sched-strategy=iterative-ilp "$@" -c fpf_wave.hip -o $out/fpf_wave.o
objs=""
for o in fpf_api fpf_generic fpf_tiled fpf_rtc fpf_selftest fpf_wblk fpf_wcoop fpf_layout fpf_vvc fpf_multi fpf_areas fpf_areas_kernels fpf_vvc_grad fpf_vvc_gradb; do objs="$objs ../lib/$o.o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libfreedm_pf.so $out/fpf_wave.o $objs -lhiprtc -lrccl -ldl
echo "$out/libfreedm_pf.so"
