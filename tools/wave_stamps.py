"""Diagnostic: per-stage cycle split of the wave kernel from the stamps build
(freedm_amd/lib/libfreedm_pf_stamps.so, `make -C freedm_amd/csrc stamps`).
Shares only -- the stamp build's own timing is not quoted (cdna_hip_programming.md 7).

Stamps (fpf_wave.hip WSTAMP, [64 waves][128]): 0 entry, 1 loads/tables staged,
2 Sld set up, 4 + 8 it + k inside sweep it (k: 0 top, 1 backward scan, 2 Ib
gathered, 3 convergence, 4 drops, 5 forward scan + stores, 6 block offsets,
7 V), 120 after the loop, 121 V written out.

    NN=123 B=4096 FPF_WAVE_GEOM=2,4 python tools/wave_stamps.py
    NN=123 B=131072 LAYOUT=1 MODEL=hosting BASE=16384 python tools/wave_stamps.py   (config 4, steady state)

BASE: the first recorded wave (global wave index, blockIdx * waves per workgroup
+ wave); the entry stamps of the recorded waves (relative to the earliest) show
how the launch's rounds line up.
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

from freedm_amd import PowerFlow, hosting_loads, scenario_loads, synthetic_feeder, _lib  # noqa: E402


def main():
    nn = int(os.environ.get("NN", "123"))
    B = int(os.environ.get("B", "4096"))
    layout = int(os.environ.get("LAYOUT", "0"))
    base = int(os.environ.get("BASE", "0"))
    f = synthetic_feeder(nn, nn)
    L = _lib.load()
    L.fpf_debug_set_wave_stamp_buffer.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = torch.zeros(64 * 128, dtype=torch.int64, device="cuda")
    pf = PowerFlow(f, kernel="wave", layout=layout)
    loads = hosting_loads if os.environ.get("MODEL") == "hosting" else scenario_loads
    pq = torch.empty((6, f.nl, B), dtype=torch.float64, device="cuda")
    for a in range(0, B, 16384):
        pq[:, :, a:a + 16384] = torch.from_numpy(loads(f, np.arange(a, min(B, a + 16384)))).cuda()
    sh = (3, pf.nn, B)
    if layout == 1:
        pq = pq.permute(2, 0, 1).contiguous()
        sh = (B, 3, pf.nn)
    out = {"loss": torch.zeros(B, dtype=torch.float64, device="cuda"),
           "iters": torch.zeros(B, dtype=torch.int32, device="cuda"),
           "status": torch.zeros(B, dtype=torch.int8, device="cuda"),
           "vmin": torch.zeros(B, dtype=torch.float64, device="cuda"),
           "vmax": torch.zeros(B, dtype=torch.float64, device="cuda"),
           "v_re": torch.zeros(sh, dtype=torch.float64, device="cuda"),
           "v_im": torch.zeros(sh, dtype=torch.float64, device="cuda")}
    for _ in range(3):
        pf.solve_device(pq, out)
    torch.cuda.synchronize()
    assert L.fpf_debug_set_wave_stamp_buffer(ctypes.c_void_p(buf.data_ptr()), base) == 0
    pf.solve_device(pq, out)
    torch.cuda.synchronize()
    st = buf.view(64, 128).cpu().numpy().astype(np.int64)
    phases = ["il+bw_scan", "ib_gather", "conv", "drops", "fw_scan+store", "blk_off", "v", "fin"]
    rows, ph, ph_it = [], [], {}
    for w in range(64):
        s = st[w]
        if s[0] == 0 or s[121] == 0:
            continue
        tops = [4 + 8 * it for it in range(12) if s[4 + 8 * it] != 0]
        n_sw = len(tops)
        d = {"staging": s[1] - s[0], "sld": s[2] - s[1], "sweeps": s[120] - s[2], "n_sweeps": n_sw,
             "v_out": s[121] - s[120], "total": s[121] - s[0]}
        if s[3]:   # (scenario-major staging: the loads landed; stamps build waits for them there)
            d["loads_landed"] = s[3] - s[0]
        if s[122] and s[123]:   # after the post-loop extremes / guard, after the barrier
            d["post_loop"] = s[122] - s[120]
            d["barrier_wait"] = s[123] - s[122]
            d["write_out"] = s[121] - s[123]
        d["per_sweep"] = d["sweeps"] / n_sw
        rows.append(d)
        for i, t in enumerate(tops):
            nxt = s[tops[i + 1]] if i + 1 < n_sw else s[120]
            marks = [s[t + k] for k in range(8)] + [nxt]
            ph.append([marks[k + 1] - marks[k] for k in range(8)])
            ph_it.setdefault(i, []).append(ph[-1])
    t0 = min(int(st[w][0]) for w in range(64) if st[w][0] != 0)
    entry = sorted(int(st[w][0]) - t0 for w in range(64) if st[w][0] != 0)
    keys = ["staging", "sld", "sweeps", "v_out", "total", "per_sweep", "n_sweeps"]
    keys += [k for k in ("loads_landed", "post_loop", "barrier_wait", "write_out") if all(k in r for r in rows)]
    mean = {k: float(np.mean([r[k] for r in rows])) for k in keys}
    phm = np.mean(np.array(ph, dtype=np.float64), axis=0)
    print(json.dumps({"nn": nn, "B": B, "layout": layout, "base": base, "entry_spread": entry[::8],
                      "tile": pf.info["tile"], "waves": len(rows), "mean_cycles": mean,
                      "share": {k: mean[k] / mean["total"] for k in ("staging", "sld", "sweeps", "v_out")},
                      "sweep_phase_cycles": {p: float(v) for p, v in zip(phases, phm)},
                      "by_sweep": {str(i): {p: round(float(v)) for p, v in zip(phases, np.mean(np.array(x, dtype=np.float64), axis=0))}
                                   for i, x in sorted(ph_it.items())}}))


if __name__ == "__main__":
    main()
