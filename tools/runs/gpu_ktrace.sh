#!/bin/bash
# rocprofv3 kernel-trace stats of short bench runs, one per "tag:dbg" in $RUNS
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in ${RUNS:-base:0}; do
  IFS=: read tag dbg <<< "$spec"
  FPF_LIB_PATH=${FPF_LIB_PATH:-} FPF_WAVE_DBG=$dbg timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$tag -o kt --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/kt_$tag.log 2>&1 || { echo "KT $tag FAILED"; tail -5 gpurun_out/kt_$tag.log; exit 1; }
  f=$(find gpurun_out/kt_$tag -name "kt_kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'dpf' in r['Name'] or 'fpf' in r['Name']:
        print('$tag', r['Name'][:60], r['Calls'], '%.1f us' % (float(r['AverageNs'])/1e3))
"
done
