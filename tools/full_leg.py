"""Diagnostic: the wave kernels' full-output variant (Vpolar / PQb / PQL, the
reference's VPQ outputs) at 4096 scenarios, scenario major: a tree feeder, the
same feeder with a zeroed phase on some laterals, and its lateral units shuffled
(the sequential-order plan); kernel time per launch (HIP events) and, for the
light outputs of the tree feeder, the same.  FPF_LIB_PATH picks the library.

    python tools/full_leg.py            (prints one JSON line)
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from freedm_amd import Feeder, PowerFlow, scenario_loads, synthetic_feeder  # noqa: E402
from lag_tables import shuffled_blocks, zeroed  # noqa: E402


def leg(f, full, B=4096, reps=10):
    dev = torch.device("cuda:0")
    pq = scenario_loads(f, np.arange(B), seed=B + 3)
    d = torch.from_numpy(np.ascontiguousarray(pq.transpose(2, 0, 1))).to(dev)
    pf = PowerFlow(f, layout=1)
    nn = pf.nn
    out = {"iters": torch.zeros(B, dtype=torch.int32, device=dev), "status": torch.zeros(B, dtype=torch.int8, device=dev),
           "loss": torch.zeros(B, dtype=torch.float64, device=dev),
           "v_re": torch.zeros((B, 3, nn), dtype=torch.float64, device=dev),
           "v_im": torch.zeros((B, 3, nn), dtype=torch.float64, device=dev)}
    if full:
        for k in ("vpolar", "pqb", "pql"):
            out[k] = torch.zeros((B, 6, nn), dtype=torch.float64, device=dev)
    for _ in range(3):
        pf.solve_device(d, out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        pf.solve_device(d, out)
    e1.record()
    torch.cuda.synchronize()
    r = {"feeder": f.name, "kernel": pf.kernel, "full": full, "ms": e0.elapsed_time(e1) / reps,
         "mean_sweeps": float(out["iters"].double().mean().item()), "n_conv": int((out["status"] == 0).sum().item())}
    pf.close()
    return r


def main():
    f = synthetic_feeder(123, 123)
    rows = [leg(f, False), leg(f, True), leg(zeroed(f), True), leg(shuffled_blocks(f, 1), True)]
    g = synthetic_feeder(2048, 2048)   # the wave-block kernel
    rows += [leg(g, False, B=2048, reps=3), leg(g, True, B=2048, reps=3), leg(zeroed(g), True, B=2048, reps=3)]
    print(json.dumps({"lib": os.environ.get("FPF_LIB_PATH", "default"), "legs": rows}))


if __name__ == "__main__":
    main()
