"""Diagnostic: where the paired wave-block kernel's time goes, from the stamps
build (freedm_amd/lib/libfreedm_pf_stamps.so, `make -C freedm_amd/csrc stamps`;
fpf_wcoop.hip CSTAMP).  64 workgroups from the middle of the grid (32 scenario
pairs) of the 4096-bus x 16384 batch: per stage, the mean share of a workgroup's
lifetime, and the per-sweep split.  Shares only (the stamps perturb timing).

Stamps [64][128]: 0 entry, 1 staged, 2 area acquired, 4 + 8 it + k in sweep it
(k: 0 top, 1 backward scan, 2 backward exchange, 3 drops, 4 forward scan,
5 forward exchange, 6 V), 120 after the loop, 121 workgroup 0's final wait.
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
    f = synthetic_feeder(4096, 4096)
    B = 16384
    base_wg = int(os.environ.get("BASE", "16384"))   # a multiple of 16: whole pairs
    L = _lib.load()
    L.fpf_debug_set_coop_stamp_buffer.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    buf = torch.zeros(64 * 128, dtype=torch.int64, device="cuda")
    pq = np.ascontiguousarray(scenario_loads(f, np.arange(512), seed=16384)[:, :, np.arange(B) % 512])
    pf = PowerFlow(f)
    assert pf.kernel == "wave" and pf.info["tile"] == 1
    pf.solve(pq, full=False)
    assert L.fpf_debug_set_coop_stamp_buffer(ctypes.c_void_p(buf.data_ptr()), base_wg) == 0
    r = pf.solve(pq, full=False)
    torch.cuda.synchronize()
    st = buf.cpu().numpy().reshape(64, 128).astype(np.float64)
    life = st[:, 120] - st[:, 0]
    out = {"wgs": 64, "base_wg": base_wg, "mean_life_cycles": float(life.mean())}
    sh = {"stage": (st[:, 1] - st[:, 0]) / life, "acquire": (st[:, 2] - st[:, 1]) / life}
    sweeps = {k: [] for k in ("bscan", "bexch", "drops", "fscan", "fexch", "v", "il_next")}
    for w in range(64):
        s = (w // 16) * 8 + (w % 8) + (base_wg // 16) * 8
        n = int(min(r["iters"][s], 14))
        for it in range(n):
            b = 4 + 8 * it
            t = st[w, b:b + 7]
            for j, k in enumerate(("bscan", "bexch", "drops", "fscan", "fexch", "v")):
                sweeps[k].append((t[j + 1] - t[j]) / life[w])
            if it + 1 < n:
                sweeps["il_next"].append((st[w, b + 8] - t[6]) / life[w])
    out["share"] = {k: float(v.mean()) for k, v in sh.items()}
    out["share_sum_over_sweeps"] = {k: float(np.sum(v) / 64) for k, v in sweeps.items()}
    out["final_wait_wg0"] = float(np.mean([(st[w, 121] - st[w, 120]) / life[w] for w in range(64) if (w // 8) % 2 == 0]))
    out["mean_sweeps"] = float(r["iters"][:B].mean())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
