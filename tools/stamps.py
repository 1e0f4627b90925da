"""Diagnostic: per-stage cycle split of the tiled kernel from the stamps build
(freedm_amd/lib/libfreedm_pf_stamps.so, `make -C freedm_amd/csrc stamps`).
Shares only -- the stamp build's own timing is not quoted (cdna_hip_programming.md 7)."""
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
    tile = int(os.environ.get("TILE", "0"))
    f = synthetic_feeder(nn, nn)
    L = _lib.load()
    L.fpf_debug_set_stamp_buffer.argtypes = [ctypes.c_void_p]
    L.fpf_debug_set_rtc_stamp_buffer.argtypes = [ctypes.c_void_p]
    spec = os.environ.get("SPEC", "1") == "1"
    buf = torch.zeros(64 * 128, dtype=torch.int64, device="cuda")
    pf = PowerFlow(f, tile=tile, specialize=spec)
    pq = torch.from_numpy(scenario_loads(f, np.arange(B))).cuda()
    out = {"loss": torch.zeros(B, dtype=torch.float64, device="cuda"),
           "iters": torch.zeros(B, dtype=torch.int32, device="cuda")}
    pf.solve_device(pq, out)
    torch.cuda.synchronize()
    assert L.fpf_debug_set_stamp_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
    assert L.fpf_debug_set_rtc_stamp_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
    pf.solve_device(pq, out)
    torch.cuda.synchronize()
    st = buf.view(64, 128).cpu().numpy().astype(np.int64)
    iters = int(out["iters"].max().item())
    names = ["P1", "S1", "P2", "S2"]
    rows = []
    for b in range(64):
        s = st[b]
        if s[0] == 0:
            continue
        d = {"init": s[1] - s[0], "total": s[127] - s[0], "epi": s[127] - s[126]}
        it = 0
        while it < 24 and s[2 + it * 5] != 0:
            prev = s[1] if it == 0 else s[5 + (it - 1) * 5]
            cur = [s[2 + it * 5 + q] for q in range(4)]
            seg = [cur[0] - prev] + [cur[q] - cur[q - 1] for q in range(1, 4)]
            for nme, v in zip(names, seg):
                d[nme] = d.get(nme, 0) + v
            it += 1
        rows.append(d)
    names = names + ["epi"]
    keys = ["init"] + names + ["total"]
    mean = {k: float(np.mean([r[k] for r in rows])) for k in keys}
    print(json.dumps({"nn": nn, "B": B, "tile": pf.info["tile"], "specialized": pf.info["specialized"], "iters": iters, "blocks": len(rows),
                      "mean_cycles": mean,
                      "share": {k: mean[k] / mean["total"] for k in keys if k != "total"}}))


if __name__ == "__main__":
    main()
