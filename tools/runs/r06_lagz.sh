#!/bin/bash
# Sequential-order tables with zeroed phases on the wave kernel (GX 3): the lag,
# wave and parity GPU tests, then the bench's sequential-order diagnostic leg.
set -o pipefail
O=gpurun_out/r06_lagz
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_lag.py tests/test_gpu_wave.py tests/test_gpu_parity.py tests/test_gpu_wblk.py -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
if [ $rc -ne 0 ]; then echo "TESTS FAILED rc=$rc"; exit $rc; fi
timeout -k 10 400 python3 -c "
import json, torch, bench
dev = torch.device('cuda:0'); torch.cuda.set_device(dev)
r = bench._diag_sequential_order(torch, 0, torch.cuda.current_stream(dev), dev)
print(json.dumps(r))" > $O/diag.json 2> $O/diag.err || { echo "DIAG FAILED"; tail -5 $O/diag.err; exit 1; }
python3 -c "
import json
d = json.load(open('$O/diag.json'))
for k, v in d.items(): print(k, v['kernel'], round(v['kernel_ms'], 4), 'exact', v['exact_kernel'], round(v['exact_kernel_ms'], 4), 'x', round(v['speedup_vs_exact'], 1), v['iters_equal_exact'], v['status_equal_exact'], v['max_v_rel_diff_vs_exact'])"
echo done
