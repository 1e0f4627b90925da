"""Per-area sweeps of every outer iteration of one config-5 solve
(FPF_AREAS_DEBUG=1; the output goes to stderr)."""
import os
import sys

os.environ["FPF_AREAS_DEBUG"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from freedm_amd import AreaPowerFlow, scenario_loads, synthetic_feeder  # noqa: E402
from freedm_amd.feeder import subtree_node_areas  # noqa: E402

f = synthetic_feeder(123, 123)
pq = scenario_loads(f, np.arange(4096), seed=4096)
ap = AreaPowerFlow(f, subtree_node_areas(f, [30, 60]), device=0)
r = ap.solve(pq, tol=1e-12, v_out=False)
print("outer", int(r["iters"].max()), r["note"], flush=True)
