"""Bitwise A/B of the batched VVC rounds between two library builds
(FPF_LIB_PATH): prints, per config-1 feeder, a digest of g, the step losses up
to each stop and the decisions of fpf_vvc_round_batch over 64 scenarios, and
its time (best of 3)."""
import hashlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from freedm_amd import PowerFlow  # noqa: E402

for name, f in bench.config1_feeders():
    pq = bench.round_scenarios(f, 64)
    pf = PowerFlow(f, device=0)
    r = pf.vvc_round_batch(f.Dl, pq)
    tt = []
    for _ in range(3):
        t0 = time.perf_counter()
        r = pf.vvc_round_batch(f.Dl, pq)
        tt.append(time.perf_counter() - t0)
    h = hashlib.sha256()
    for s in range(64):
        for x in range(3):
            h.update(np.ascontiguousarray(r["g"][s][x]).tobytes())
        st = int(r["stop_fwd"][s])
        h.update(np.ascontiguousarray(r["loss_fwd"][s, : (st + 2 if st >= 0 else 101)]).tobytes())
    for k in ("stop_fwd", "stop_rev", "reversed", "sent"):
        h.update(np.asarray(r[k]).tobytes())
    print(f"{name}: {min(tt) * 1e3:.3f} ms digest {h.hexdigest()[:16]}", flush=True)
    pf.close()
