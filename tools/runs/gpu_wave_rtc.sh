#!/bin/bash
# The per-plan hipRTC wave / wave-block kernels against the static ones on the
# same box: their GPU tests, then the default bench line (configs 2 and 4) and
# config 3 alternating specialised / static (--no-specialize).  gpurun_out/$P.
set -o pipefail
P=${P:-r04rtc}
mkdir -p gpurun_out/$P
export TMPDIR=/tmp
export FPF_WAVE_RTC=${FPF_WAVE_RTC:-2048}
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_wave.py tests/test_gpu_wblk.py tests/test_rtc_compile.py -x -v --timeout 150 --timeout-method thread > gpurun_out/$P/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/$P/pytest.log; exit 1; }
tail -2 gpurun_out/$P/pytest.log
summ() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; r4=d.get("roofline_config4"); a=d.get("config5_areas"); print("kernel_ms %.5f frac %.4f rtc %s" % (r["kernel_ms"], r["frac"], d["config"].get("wave_rtc_builds")), ("| c4 kernel_ms %.4f frac %.4f | c5 %.3fx" % (r4["kernel_ms"], r4["frac"], a["vs_monolithic"])) if r4 else "")'; }
for rep in 1 2; do
  for sp in spec static; do
    A=""; [ $sp = static ] && A="--no-specialize"
    timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline $A > gpurun_out/$P/bench_${sp}_$rep.log 2>&1 || { echo "BENCH $sp FAILED"; tail -30 gpurun_out/$P/bench_${sp}_$rep.log; exit 1; }
    echo "c2/c4 $sp $rep: $(tail -1 gpurun_out/$P/bench_${sp}_$rep.log | summ 2>&1 | cut -c1-300)"
    timeout -k 10 300 python3 -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline $A > gpurun_out/$P/bench_c3_${sp}_$rep.log 2>&1 || { echo "C3 $sp FAILED"; tail -30 gpurun_out/$P/bench_c3_${sp}_$rep.log; exit 1; }
    echo "c3 $sp $rep: $(tail -1 gpurun_out/$P/bench_c3_${sp}_$rep.log | summ 2>&1 | cut -c1-300)"
  done
done
for sch in wave wblk; do
  V=$(echo $sch | tr a-z A-Z)
  env FPF_${V}_RTC_SCHED=0 timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/$P/bench_dflt_$sch.log 2>&1 || { echo "BENCH dflt FAILED"; exit 1; }
  echo "c2/c4 default-sched $sch: $(tail -1 gpurun_out/$P/bench_dflt_$sch.log | summ 2>&1 | cut -c1-300)"
  env FPF_${V}_RTC_SCHED=0 timeout -k 10 300 python3 -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/$P/bench_c3_dflt_$sch.log 2>&1 || { echo "C3 dflt FAILED"; exit 1; }
  echo "c3 default-sched $sch: $(tail -1 gpurun_out/$P/bench_c3_dflt_$sch.log | summ 2>&1 | cut -c1-300)"
done
echo DONE
