"""The bench's config-1 batched-round leg alone for one feeder (rocprofv3 traces
it): B whole VVC rounds via fpf_vvc_round_batch, timed best of 3."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from freedm_amd import PowerFlow  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "123bus"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
f = dict(bench.config1_feeders())[name]
pq = bench.round_scenarios(f, B)
pf = PowerFlow(f, device=0)
pf.vvc_round_batch(f.Dl, pq)
tt = []
for _ in range(3):
    t0 = time.perf_counter()
    r = pf.vvc_round_batch(f.Dl, pq)
    tt.append(time.perf_counter() - t0)
print({"feeder": name, "B": B, "ms": min(tt) * 1e3, "n_bad": int(r["n_bad"]), "reversed": int(r["reversed"].sum())})
