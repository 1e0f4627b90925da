"""Diagnostic: per-stage cycle split of the wave kernel from the stamps build
(freedm_amd/lib/libfreedm_pf_stamps.so, `make -C freedm_amd/csrc stamps`).
Shares only -- the stamp build's own timing is not quoted (cdna_hip_programming.md 7).

Stamps (fpf_wave.hip WSTAMP, [64 waves][128]): 0 entry, 1 loads/tables staged,
2 Sld set up, 4 + 8 it + k inside sweep it (k: 0 top, 1 backward scan, 2 Ib
gathered, 3 convergence, 4 drops, 5 forward scan + stores, 6 block offsets,
7 V), 120 after the loop, 121 V written out.

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
    buf = torch.zeros(64 * 128, dtype=torch.int64, device="cuda")
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
    st = buf.view(64, 128).cpu().numpy().astype(np.int64)
    phases = ["il+bw_scan", "ib_gather", "conv", "drops", "fw_scan+store", "blk_off", "v", "fin"]
    rows, ph = [], []
    for w in range(64):
        s = st[w]
        if s[0] == 0 or s[121] == 0:
            continue
        tops = [4 + 8 * it for it in range(12) if s[4 + 8 * it] != 0]
        n_sw = len(tops)
        d = {"staging": s[1] - s[0], "sld": s[2] - s[1], "sweeps": s[120] - s[2], "n_sweeps": n_sw,
             "v_out": s[121] - s[120], "total": s[121] - s[0]}
        d["per_sweep"] = d["sweeps"] / n_sw
        rows.append(d)
        for i, t in enumerate(tops):
            nxt = s[tops[i + 1]] if i + 1 < n_sw else s[120]
            marks = [s[t + k] for k in range(8)] + [nxt]
            ph.append([marks[k + 1] - marks[k] for k in range(8)])
    keys = ["staging", "sld", "sweeps", "v_out", "total", "per_sweep", "n_sweeps"]
    mean = {k: float(np.mean([r[k] for r in rows])) for k in keys}
    phm = np.mean(np.array(ph, dtype=np.float64), axis=0)
    print(json.dumps({"nn": nn, "B": B, "tile": pf.info["tile"], "waves": len(rows), "mean_cycles": mean,
                      "share": {k: mean[k] / mean["total"] for k in ("staging", "sld", "sweeps", "v_out")},
                      "sweep_phase_cycles": {p: float(v) for p, v in zip(phases, phm)}}))


if __name__ == "__main__":
    main()
