"""Diagnostic: per-stage cycle split of the wave kernel from the stamps build
(freedm_amd/lib/libfreedm_pf_stamps.so, `make -C freedm_amd/csrc stamps`).
Shares only -- the stamp build's own timing is not quoted (cdna_hip_programming.md 7).

    NN=123 B=4096 FPF_WAVE_GEOM=2,4 python tools/wave_stamps.py
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["FPF_LIB_PATH"] = os.path.join(ROOT, "freedm_amd", "lib", "libfreedm_pf_stamps.so")

import torch  # noqa: E402

from freedm_amd import PowerFlow, scenario_loads, synthetic_feeder, _lib  # noqa: E402

STAGES = ["IL", "bw_scan", "bw_gather", "drop", "fw_scan", "fw_resolve_V"]


def main():
    nn = int(os.environ.get("NN", "123"))
    B = int(os.environ.get("B", "4096"))
    f = synthetic_feeder(nn, nn)
    L = _lib.load()
    L.fpf_debug_set_wave_stamp_buffer.argtypes = [ctypes.c_void_p]
    buf = torch.zeros(64 * 64, dtype=torch.int64, device="cuda")
    pf = PowerFlow(f, kernel="wave")
    pq = torch.from_numpy(scenario_loads(f, np.arange(B))).cuda()
    out = {"loss": torch.zeros(B, dtype=torch.float64, device="cuda"),
           "iters": torch.zeros(B, dtype=torch.int32, device="cuda")}
    for _ in range(3):
        pf.solve_device(pq, out)
    torch.cuda.synchronize()
    assert L.fpf_debug_set_wave_stamp_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
    pf.solve_device(pq, out)
    torch.cuda.synchronize()
    st = buf.view(64, 64).cpu().numpy().astype(np.int64)
    rows = []
    for w in range(64):
        s = st[w]
        if s[0] == 0 or s[1] == 0:
            continue
        d = {"init": s[1] - s[0], "epi": 0}
        it = 0
        prev = s[1]
        while it < 9 and s[2 + 6 * it] != 0 and s[7 + 6 * it] != 0:
            for q, nme in enumerate(STAGES):
                cur = s[2 + 6 * it + q]
                d[nme] = d.get(nme, 0) + (cur - prev)
                prev = cur
            it += 1
        d["sweeps"] = it
        d["total"] = prev - s[0]
        rows.append(d)
    keys = ["init"] + STAGES + ["total"]
    mean = {k: float(np.mean([r.get(k, 0) for r in rows])) for k in keys}
    print(json.dumps({"nn": nn, "B": B, "geom": [pf.info["tile"]], "waves": len(rows),
                      "sweeps": float(np.mean([r["sweeps"] for r in rows])),
                      "mean_cycles": mean, "share": {k: mean[k] / mean["total"] for k in keys if k != "total"}}))


if __name__ == "__main__":
    main()
