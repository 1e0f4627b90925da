#!/bin/bash
# The config-5 leg (tools/c5_leg.py) under each schedule ($MODES: "tag:ENV=..,ENV=.."),
# then a rocprofv3 kernel trace of the default (the timeline: tools/c5_timeline.py)
set -o pipefail
TAG=${TAG:-c5}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
for spec in ${MODES:-default:}; do
  IFS=: read tag envs <<< "$spec"
  env ${envs//,/ } timeout -k 10 180 python3 -u tools/c5_leg.py > gpurun_out/$TAG/leg_$tag.log 2>&1 || { tail -5 gpurun_out/$TAG/leg_$tag.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/$TAG/leg_$tag.log)"
done
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/$TAG/kt -o kt --output-format csv -- python3 tools/c5_leg.py \
  > gpurun_out/$TAG/kt.log 2>&1 || { tail -5 gpurun_out/$TAG/kt.log; exit 1; }
tail -1 gpurun_out/$TAG/kt.log
