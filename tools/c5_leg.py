"""The bench's config-5 leg alone (tools/runs/gpu_r03n.sh profiles it): the 123-bus
feeder in 3 areas, one config-2 batch, host buffers, tolerance 1e-12."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from freedm_amd import AreaPowerFlow, PowerFlow, scenario_loads, synthetic_feeder  # noqa: E402
from freedm_amd.feeder import subtree_node_areas  # noqa: E402

f = synthetic_feeder(123, 123)
pq = scenario_loads(f, np.arange(4096), seed=4096)
pf = PowerFlow(f, device=0)
pf.solve(pq, full=False)
th = []
for _ in range(5):
    t0 = time.perf_counter()
    pf.solve(pq, full=False)
    th.append(time.perf_counter() - t0)
ap = AreaPowerFlow(f, subtree_node_areas(f, [30, 60]), device=0)
ap.solve(pq, tol=1e-12, v_out=False)
ta = []
for _ in range(5):
    t0 = time.perf_counter()
    r = ap.solve(pq, tol=1e-12, v_out=False)
    ta.append(time.perf_counter() - t0)
print({"mono_ms": min(th) * 1e3, "areas_ms": min(ta) * 1e3, "ratio": min(ta) / min(th), "outer": int(r["iters"].max()),
       "area_nodes": ap.area_nodes})
