#!/bin/bash
# Round 5: wave-block offsets per (block, phase) -- parity, then config 3 and the
# trimmed timed region (config 2 at K = 20, one and two streams)
set -o pipefail
OUT=gpurun_out/r05c3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_wblk.py tests/test_gpu_wcoop.py > $OUT/pytest.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAIL|Error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  timeout -k 10 300 python3 -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/c3_r$rep.log 2>&1 || { echo "C3 FAILED"; tail -20 $OUT/c3_r$rep.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$OUT/c3_r$rep.log') if l.startswith('{')][-1])
print('c3 r$rep kernel_ms %.4f frac %.4f n_conv %d' % (d['roofline']['kernel_ms'], d['roofline']['frac'], d['aggregate']['n_conv']))"
done
for S in 1 2; do
  FPF_BENCH_TRACE=1 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c4 --streams $S > $OUT/c2_s$S.log 2> $OUT/c2_s$S.err || { echo "C2 FAILED"; tail -20 $OUT/c2_s$S.err; exit 1; }
  grep timed_study $OUT/c2_s$S.err
  python3 -c "
import json; d=json.loads([l for l in open('$OUT/c2_s$S.log') if l.startswith('{')][-1])
print('c2 S=$S value %.1f M/s ms_per_step %.4f kernel_ms %.4f' % (d['value']/1e6, d['ms_per_step'], d['roofline']['kernel_ms']))"
done
