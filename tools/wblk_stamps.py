"""Diagnostic: where the wave-block kernel's time goes (config 3: 2048-bus x
65 536, scenario major), from the stamps build (freedm_amd/lib/
libfreedm_pf_stamps.so, `make -C freedm_amd/csrc stamps`; fpf_wblk_body.h
BSTAMP).  64 workgroups from BASE on (steady state): per stage the mean cycles
of a workgroup's lifetime and the per-sweep split.  The stamps build runs the
static kernel (the default scheduler) and its own stamp stores: shares, not
absolute times.

Stamps [64][128]: 0 entry, 1 staged, 4 + 8 it + k in sweep it (k: 0 top,
1 backward scan + totals, 2 Ib gathered, 3 drops, 4 forward scan + totals,
5 block offsets, 6 V), 120 after the loop, 121 extremes, 122 results, 123 V out.
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
    nn = int(os.environ.get("NN", "2048"))
    B = int(os.environ.get("B", "65536"))
    base = int(os.environ.get("BASE", "32768"))
    f = synthetic_feeder(nn, nn)
    L = _lib.load()
    L.fpf_debug_set_wblk_stamp_buffer.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    buf = torch.zeros(64 * 128, dtype=torch.int64, device="cuda")
    pf = PowerFlow(f, layout=1)
    assert pf.kernel == "wave" and pf.info["tile"] == 1
    pq = torch.empty((B, 6, f.nl), dtype=torch.float64, device="cuda")
    for a in range(0, B, 4096):
        pq[a:a + 4096] = torch.from_numpy(np.ascontiguousarray(
            scenario_loads(f, np.arange(a, min(B, a + 4096)), seed=65536).transpose(2, 0, 1))).cuda()
    out = {"loss": torch.zeros(B, dtype=torch.float64, device="cuda"),
           "iters": torch.zeros(B, dtype=torch.int32, device="cuda"),
           "status": torch.zeros(B, dtype=torch.int8, device="cuda"),
           "vmin": torch.zeros(B, dtype=torch.float64, device="cuda"),
           "vmax": torch.zeros(B, dtype=torch.float64, device="cuda"),
           "v_re": torch.zeros((B, 3, pf.nn), dtype=torch.float64, device="cuda"),
           "v_im": torch.zeros((B, 3, pf.nn), dtype=torch.float64, device="cuda")}
    pf.solve_device(pq, out)
    torch.cuda.synchronize()
    assert L.fpf_debug_set_wblk_stamp_buffer(ctypes.c_void_p(buf.data_ptr()), base) == 0
    pf.solve_device(pq, out)
    torch.cuda.synchronize()
    st = buf.view(64, 128).cpu().numpy().astype(np.int64)
    it = out["iters"].cpu().numpy()
    rows, ph = [], []
    names = ["bw_scan+totals", "ib_gather", "drops", "fw_scan+totals", "blk_off", "v", "next_top"]
    for w in range(64):
        s = st[w]
        if s[0] == 0 or s[123] == 0:
            continue
        n = int(sum(1 for k in range(14) if s[4 + 8 * k] != 0))
        rows.append({"staging": s[1] - s[0], "to_loop": s[4] - s[1], "sweeps": s[120] - s[4], "n_sweeps": n,
                     "extremes": s[121] - s[120], "results": s[122] - s[121], "v_out": s[123] - s[122],
                     "total": s[123] - s[0]})
        for k in range(n):
            t = [s[4 + 8 * k + j] for j in range(7)]
            nxt = s[4 + 8 * (k + 1)] if k + 1 < n else s[120]
            ph.append([t[j + 1] - t[j] for j in range(6)] + [nxt - t[6]])
    keys = ["staging", "to_loop", "sweeps", "extremes", "results", "v_out", "total", "n_sweeps"]
    mean = {k: float(np.mean([r[k] for r in rows])) for k in keys}
    mean["per_sweep"] = mean["sweeps"] / mean["n_sweeps"]
    phm = np.mean(np.array(ph, dtype=np.float64), axis=0)
    print(json.dumps({"nn": nn, "B": B, "base": base, "wgs": len(rows), "mean_cycles": mean,
                      "share": {k: mean[k] / mean["total"] for k in keys[:6]},
                      "sweep_phase_cycles": {p: float(v) for p, v in zip(names, phm)},
                      "mean_iters_batch": float(it.mean())}))


if __name__ == "__main__":
    main()
