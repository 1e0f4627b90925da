#!/bin/bash
# One GPU-box pass: smoke -> GPU parity tests -> short bench.  Every GPU step has
# its own time limit and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
(nproc; lscpu | grep -E "Model name|^CPU\(s\)"; rocminfo 2>/dev/null | grep -E "Marketing Name|Name: +gfx" | head -4) > gpurun_out/box.txt 2>&1
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAILED rc=$?"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 30 --warmup 5 --cpu-seconds 5 > gpurun_out/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
