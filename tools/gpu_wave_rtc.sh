#!/bin/bash
# The per-plan hipRTC wave kernel against the static one on the same box: its
# GPU tests, then the default bench line (configs 2 and 4) alternating
# specialised / static (--no-specialize).  Everything under gpurun_out/$P.
set -o pipefail
P=${P:-r04rtc}
mkdir -p gpurun_out/$P
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_wave.py tests/test_rtc_compile.py -x -v --timeout 120 --timeout-method thread > gpurun_out/$P/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/$P/pytest.log; exit 1; }
tail -2 gpurun_out/$P/pytest.log
for rep in 1 2; do
  for sp in spec static; do
    A=""; [ $sp = static ] && A="--no-specialize"
    timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline $A > gpurun_out/$P/bench_${sp}_$rep.log 2>&1 || { echo "BENCH $sp FAILED"; tail -30 gpurun_out/$P/bench_${sp}_$rep.log; exit 1; }
    echo "$sp $rep: $(tail -1 gpurun_out/$P/bench_${sp}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; r4=d["roofline_config4"]; a=d["config5_areas"]; print("c2 kernel_ms %.5f frac %.4f | c4 kernel_ms %.4f frac %.4f | c5 %.3f x" % (r["kernel_ms"], r["frac"], r4["kernel_ms"], r4["frac"], a["vs_monolithic"]))' 2>&1 | cut -c1-400)"
  done
done
echo DONE
