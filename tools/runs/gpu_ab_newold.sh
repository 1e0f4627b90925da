set -o pipefail
mkdir -p gpurun_out/ab2
timeout -k 10 600 python -u -m pytest tests/test_gpu_layout.py tests/test_gpu_wblk.py tests/test_gpu_parity.py tests/test_gpu_wave.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab2/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/ab2/pytest.log; exit 1; }
tail -2 gpurun_out/ab2/pytest.log
VARIANTS="new:- old:FPF_LIB_PATH=freedm_amd/lib/abl/libfreedm_pf_old.so" bash tools/runs/gpu_ab.sh || exit 1
for V in new old; do
  if [ $V = old ]; then export FPF_LIB_PATH=freedm_amd/lib/abl/libfreedm_pf_old.so; else unset FPF_LIB_PATH; fi
  timeout -k 10 200 python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab2/c3_$V.json 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab2/c3_$V.json').readlines()[-1]); print('$V c3', d['roofline']['kernel_ms'])"
done
