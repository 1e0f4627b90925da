#!/bin/bash
# A/B of environment variants on the bench (config 2 + config-4 roofline), each
# run twice, alternating: VARIANTS="name:ENV=val+ENV2=val name2:..." ("-" = none)
set -o pipefail
mkdir -p gpurun_out/ab
for rep in 1 2; do
for V in $VARIANTS; do
  name=${V%%:*}; envs=${V#*:}
  [ "$envs" = "-" ] && envs=""
  env ${envs//+/ } timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab/${name}_$rep.log 2>&1 || { echo "FAILED $name"; tail -5 gpurun_out/ab/${name}_$rep.log; exit 1; }
  python3 - gpurun_out/ab/${name}_$rep.log $name <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r, r4 = d["roofline"], d.get("roofline_config4", {})
print("%-12s c2 %.4f ms | c4 %.4f ms | conv %d" % (sys.argv[2], r["kernel_ms"], r4.get("kernel_ms", 0), d["aggregate"]["n_conv"]))
PY
done
done
