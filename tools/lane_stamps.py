"""Diagnostic: where the lane kernel's time goes (config 4: 131 072 hosting
scenarios of the 123-bus feeder, scenario-fastest), from its stamps build
(`tools/build_lane_variants.sh stamps=-DFPF_LANE_STAMPS`; fpf_lane.hip LSTAMP).
The 64 waves of eight workgroups from BASE on record s_memtime at the phase
boundaries of every sweep; printed: mean cycles per phase of a sweep (barrier
waits separately) and the shares of a wave's lifetime.  The stamps' own stores
and waits perturb the kernel: shares, not absolute times.

Stamps [64][128]: 0 entry, 1 loop start, 4 + 10 it + k in sweep it (k: 0 top,
1 currents, 2 B1, 3 carry + E published, 4 B2, 5 drops, 6 B3, 7 G published,
8 B4, 9 voltages), 120 after the loop, 121 V out, 122 end.
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FPF_LIB_PATH", os.path.join(ROOT, "freedm_amd", "lib", "abl", "libfreedm_pf_lane_stamps.so"))
os.environ.setdefault("FPF_LANE", "1")

import torch  # noqa: E402

from freedm_amd import PowerFlow, hosting_loads, synthetic_feeder, _lib  # noqa: E402

NAMES = ["currents", "B1 wait", "carry+publish E", "B2 wait", "drops", "B3 wait", "publish G", "B4 wait", "voltages"]


def main():
    B = int(os.environ.get("B", "131072"))
    base = int(os.environ.get("BASE", "1024"))
    f = synthetic_feeder(123, 123)
    L = _lib.load()
    L.fpf_debug_set_lane_stamp_buffer.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    buf = torch.zeros(64 * 128, dtype=torch.int64, device="cuda")
    pf = PowerFlow(f, layout=0)
    pq = torch.empty((6, f.Dl.shape[0], B), dtype=torch.float64, device="cuda")
    for a in range(0, B, 16384):
        pq[:, :, a:a + 16384] = torch.from_numpy(hosting_loads(f, np.arange(a, min(B, a + 16384)), seed=1 << 20)).cuda()
    out = {k: torch.zeros(B, dtype=torch.float64, device="cuda") for k in ("loss", "vmin", "vmax")}
    out["iters"] = torch.zeros(B, dtype=torch.int32, device="cuda")
    out["status"] = torch.zeros(B, dtype=torch.int8, device="cuda")
    out["v_re"] = torch.zeros((3, pf.nn, B), dtype=torch.float64, device="cuda")
    out["v_im"] = torch.zeros((3, pf.nn, B), dtype=torch.float64, device="cuda")
    n0 = L.fpf_lane_launches()
    pf.solve_device(pq, out)
    torch.cuda.synchronize()
    assert L.fpf_debug_set_lane_stamp_buffer(ctypes.c_void_p(buf.data_ptr()), base) == 0
    pf.solve_device(pq, out)
    torch.cuda.synchronize()
    assert L.fpf_lane_launches() == n0 + 2, "the lane kernel did not run"
    st = buf.view(64, 128).cpu().numpy().astype(np.int64)
    ph, life = [], []
    for w in range(64):
        s = st[w]
        if s[0] == 0 or s[122] == 0:
            continue
        n = int(sum(1 for k in range(12) if s[4 + 10 * k] != 0))
        for k in range(n):
            t = [s[4 + 10 * k + j] for j in range(10)]
            ph.append([t[j + 1] - t[j] for j in range(9)])
        life.append({"setup": s[1] - s[0], "sweeps": s[120] - s[1], "v_out": s[121] - s[120],
                     "results": s[122] - s[121], "total": s[122] - s[0], "n_sweeps": n})
    phm = np.mean(np.array(ph, dtype=np.float64), axis=0)
    lm = {k: float(np.mean([r[k] for r in life])) for k in life[0]}
    print(json.dumps({"B": B, "base": base, "waves": len(life), "mean_cycles": lm,
                      "per_sweep_cycles": float(phm.sum()),
                      "sweep_phase_cycles": {p: round(float(v), 1) for p, v in zip(NAMES, phm)},
                      "sweep_phase_share": {p: round(float(v / phm.sum()), 3) for p, v in zip(NAMES, phm)}}))


if __name__ == "__main__":
    main()
