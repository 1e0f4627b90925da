"""Diagnostic: per-stage cycle split of the wave kernel from the stamps build
(freedm_amd/lib/libfreedm_pf_stamps.so, `make -C freedm_amd/csrc stamps`).
Shares only -- the stamp build's own timing is not quoted (cdna_hip_programming.md 7).

Stamps (fpf_wave.hip WSTAMP): 0 entry, 1 loads/tables staged, 2 Sld set up,
3 + it end of sweep it, 40 after the loop, 41 V written out.

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
           "iters": torch.zeros(B, dtype=torch.int32, device="cuda"),
           "v_re": torch.zeros((3, pf.nn, B), dtype=torch.float64, device="cuda"),
           "v_im": torch.zeros((3, pf.nn, B), dtype=torch.float64, device="cuda")}
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
        if s[0] == 0 or s[41] == 0:
            continue
        sw = [s[3 + i] for i in range(37) if s[3 + i] != 0]
        d = {"staging": s[1] - s[0], "sld": s[2] - s[1], "sweeps": sw[-1] - s[2], "n_sweeps": len(sw),
             "after_loop": s[40] - sw[-1], "v_out": s[41] - s[40], "total": s[41] - s[0]}
        d["per_sweep"] = d["sweeps"] / len(sw)
        rows.append(d)
    keys = ["staging", "sld", "sweeps", "after_loop", "v_out", "total", "per_sweep", "n_sweeps"]
    mean = {k: float(np.mean([r[k] for r in rows])) for k in keys}
    print(json.dumps({"nn": nn, "B": B, "tile": pf.info["tile"], "waves": len(rows), "mean_cycles": mean,
                      "share": {k: mean[k] / mean["total"] for k in ("staging", "sld", "sweeps", "after_loop",
                                                                      "v_out")}}))


if __name__ == "__main__":
    main()
