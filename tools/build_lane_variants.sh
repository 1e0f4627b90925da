#!/bin/bash
# Diagnostic builds of the lane kernel (never the product): each NAME=FLAGS pair
# compiles fpf_lane.hip with FLAGS and links it with the product's other objects
# into freedm_amd/lib/abl/libfreedm_pf_lane_NAME.so (FPF_LIB_PATH selects one).
set -e
cd "$(dirname "$0")/../freedm_amd/csrc"
make -s -j8 ../lib/libfreedm_pf.so
OBJS=$(ls ../lib/fpf_*.o | grep -v fpf_lane.o)
mkdir -p ../lib/abl
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../../include $flags -c fpf_lane.hip -o ../lib/abl/lane_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/abl/libfreedm_pf_lane_$name.so $OBJS ../lib/abl/lane_$name.o -lhiprtc -lrccl -ldl
  echo "built lane_$name ($flags)"
done
