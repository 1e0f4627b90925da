#!/bin/bash
# freedm_amd/lib/var_<name>/libfreedm_pf.so: the product library with one kernel
# source (fpf_wave, fpf_wblk, fpf_wcoop, ...) built with extra flags (experiments;
# load with FPF_LIB_PATH).   tools/build_obj_variant.sh fpf_wcoop ilp -mllvm -amdgpu-sched-strategy=iterative-ilp
set -e
src=$1; name=$2; shift 2
cd "$(dirname "$0")/../freedm_amd/csrc"
make -s -j8 >/dev/null
out=../lib/var_$name
mkdir -p $out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result -I../../include \
  "$@" -c $src.hip -o $out/$src.o
objs=""
for o in fpf_api fpf_generic fpf_tiled fpf_rtc fpf_selftest fpf_wave fpf_wblk fpf_wcoop fpf_layout fpf_vvc fpf_multi fpf_areas fpf_areas_kernels fpf_vvc_grad fpf_vvc_gradb; do
  [ "$o" = "$src" ] && objs="$objs $out/$o.o" || objs="$objs ../lib/$o.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libfreedm_pf.so $objs -lhiprtc -lrccl -ldl
echo "$out/libfreedm_pf.so"
