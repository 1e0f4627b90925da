#!/bin/bash
# A/B of whole builds on the bench (config 2 + config-4 leg, then config 3), run
# twice, alternating.  VARIANTS="name:DIR:LIB ..." -- bench.py of tree DIR ("." =
# this one) with FPF_LIB_PATH=LIB ("-" = the tree's own library).
set -o pipefail
mkdir -p gpurun_out/abt
ROOT=$(pwd)
for rep in 1 2; do
for V in $VARIANTS; do
  IFS=: read -r name dir lib <<< "$V"
  log=$ROOT/gpurun_out/abt/${name}_$rep
  ( cd "$dir" || exit 1
    if [ "$lib" != "-" ]; then export FPF_LIB_PATH=$lib; fi
    timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $log.c2.log 2>&1 || exit 1
    [ -n "$NO_C3" ] || timeout -k 10 300 python3 -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > $log.c3.log 2>&1 || exit 1
  ) || { echo "FAILED $name"; tail -5 $log.c2.log $log.c3.log 2>/dev/null; exit 1; }
  python3 - $log $name <<'PY'
import json, os, sys
def last(p):
    return json.loads([l for l in open(p) if l.startswith("{")][-1]) if os.path.exists(p) else None
d, d3 = last(sys.argv[1] + ".c2.log"), last(sys.argv[1] + ".c3.log")
r, r4 = d["roofline"], d.get("roofline_config4", {})
c3 = d3["roofline"]["kernel_ms"] if d3 else 0
print("%-8s c2 %.4f ms | c4 %.4f ms | c3 %.3f ms" % (sys.argv[2], r["kernel_ms"], r4.get("kernel_ms", 0), c3))
PY
done
done
