"""One specialised (hipRTC) wave launch against the static kernel on the GPU box:
python tools/wave_rtc_probe.py <nodes> <full 0/1> [prefull] -- light
(solve_device) or full (solve) outputs; prints whether they are identical and
the build count."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from freedm_amd import PowerFlow, _lib, feeder as F  # noqa: E402

n, full = int(sys.argv[1]), int(sys.argv[2])
prefull = len(sys.argv) > 3 and sys.argv[3] == "prefull"   # a static full-output solve first
f = F.synthetic_feeder(n, n)
B = 4096
pq = F.scenario_loads(f, np.arange(B))
if prefull:
    PowerFlow(f, kernel="wave", specialize=False).solve(pq)
    print("static full-output solve done", flush=True)
L = _lib.load()
L.fpf_wave_rtc_builds.restype = C.c_int
dev = torch.device("cuda:0")
res = []
for spec in (False, True):
    pf = PowerFlow(f, kernel="wave", specialize=spec)
    if full:
        r = pf.solve(pq)
        res.append({k: np.asarray(v) for k, v in r.items()})
    else:
        out = {"v_re": torch.zeros((3, pf.nn, B), dtype=torch.float64, device=dev),
               "v_im": torch.zeros((3, pf.nn, B), dtype=torch.float64, device=dev),
               "iters": torch.zeros(B, dtype=torch.int32, device=dev),
               "status": torch.zeros(B, dtype=torch.int8, device=dev),
               "loss": torch.zeros(B, dtype=torch.float64, device=dev)}
        pf.solve_device(torch.from_numpy(pq).to(dev), out)
        torch.cuda.synchronize()
        res.append({k: v.cpu().numpy() for k, v in out.items()})
    print("spec", spec, "builds", L.fpf_wave_rtc_builds(), flush=True)
bad = [k for k in res[0] if not np.array_equal(res[0][k], res[1][k])]
print("n", n, "full", full, "identical" if not bad else f"DIFFER {bad}", flush=True)
