"""Generate the golden fixtures under tests/golden/ (run from the repo root:
`python tests/golden/make_golden.py`).

The reference itself cannot run here (Armadillo is absent), so
the vectors come from the C oracle (oracle/ref_dpf.c) and are accepted only if
the independent NumPy restatement (oracle/np_dpf.py) agrees with them to 1e-12
relative with identical iteration counts.  Inputs are the reference's own
feeders (load_system_data's 9-row feeder, Broker/Dl_new.mat + the supplied Z)
plus seeded synthetic feeders and edge cases.
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from freedm_amd import feeder as F  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle.np_dpf import dpf_batch_np, vvc_reduce_np  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def missing_phase_feeder() -> F.Feeder:
    """G6: the 9-row feeder with a phase-B-only code on the 1->6 lateral, so
    phases A/C are zeroed there (angles read -180/+180, DPF_return7.cpp:180-192,232-235)."""
    f = F.demo_feeder()
    Z = np.vstack([f.Z, np.diag([0, 2.0 + 6.0j, 0])])
    Dl = f.Dl.copy()
    Dl[6:9, 3] = 3
    Dl[6:9, 6] = 0
    Dl[6:9, 10] = 0
    return F.Feeder(Dl, Z, name="demo-missing-phase")


def nonconvergent_feeder() -> F.Feeder:
    """G5: the 9-row feeder overloaded 40x -- no sweep meets errmx < 1e-4."""
    f = F.demo_feeder()
    Dl = f.Dl.copy()
    Dl[:, 6:12] *= 40
    return F.Feeder(Dl, f.Z, name="demo-overloaded")


def cases():
    demo = F.demo_feeder()
    yield "g1_demo", demo, demo.base_pq[:, :, None]
    yield "g1_demo_batch", demo, F.scenario_loads(demo, np.arange(32))
    dln = F.dl_new_feeder()
    yield "g2_dlnew", dln, np.concatenate([dln.base_pq[:, :, None], F.scenario_loads(dln, np.arange(31))], axis=2)
    f123 = F.synthetic_feeder(123, 123)
    yield "g3_123bus", f123, F.scenario_loads(f123, np.arange(16))
    f2048 = F.synthetic_feeder(2048, 2048)
    yield "g4_2048bus", f2048, F.scenario_loads(f2048, np.arange(2))
    nc = nonconvergent_feeder()
    yield "g5_nonconv", nc, np.concatenate([nc.base_pq[:, :, None], demo.base_pq[:, :, None]], axis=2)
    mp = missing_phase_feeder()
    yield "g6_missing_phase", mp, F.scenario_loads(mp, np.arange(8))


def main():
    for name, f, pq in cases():
        c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
        n = dpf_batch_np(f.Dl, f.Z, pq)
        ln = O.lnum(f.Dl, f.Z)
        loss, vmin, vmax = vvc_reduce_np(n["Vpolar"], n["PQb"], n["PQL"], ln)
        assert (c["iters"] == n["iters"]).all(), name
        vc = c["V_re"] + 1j * c["V_im"]
        vn = n["V_re"] + 1j * n["V_im"]
        rel = np.max(np.abs(vc - vn) / np.maximum(np.abs(vn), 1e-300))
        # a non-converging iteration amplifies last-bit differences over 20 sweeps
        assert rel < (1e-12 if (c["status"] == 0).all() else 1e-9), (name, rel)
        assert np.allclose(c["loss"], loss, rtol=1e-9, atol=1e-9), name
        assert np.allclose(c["vmin"], vmin, rtol=1e-13) and np.allclose(c["vmax"], vmax, rtol=1e-13), name
        np.savez_compressed(
            os.path.join(OUT, f"{name}.npz"),
            Dl=f.Dl, Z=f.Z, pq=pq, lnum=np.array(ln),
            iters=c["iters"], status=c["status"], loss=c["loss"], vmin=c["vmin"], vmax=c["vmax"],
            V_re=c["V_re"], V_im=c["V_im"],
            Vpolar=c["Vpolar"][:, :, :4], PQb=c["PQb"][:, :, :4], PQL=c["PQL"][:, :, :4],
        )
        print(f"{name:18s} nl={f.nl:5d} nn={f.n_nodes:5d} B={pq.shape[2]:3d} iters={np.unique(c['iters']).tolist()} "
              f"status={np.unique(c['status']).tolist()} np-vs-C V rel={rel:.1e} "
              f"size={os.path.getsize(os.path.join(OUT, name + '.npz')) // 1024} KB")


if __name__ == "__main__":
    main()
