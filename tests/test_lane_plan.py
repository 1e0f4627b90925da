"""fpf_feeder_lane_plan (no device): the lane kernel's plan (fpf_api.cpp:
analyse_lane) for the benched feeders, and a numpy re-enactment of the lane
kernel's algebra on that plan (fpf_lane.hip: wave-local prefix sums, wave
carries, published subtree ends and taps, block offsets) checked against the
oracle -- the tables and the algebra are right before any GPU runs them."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

from freedm_amd import _lib
from freedm_amd import feeder as F

sys.path.insert(0, os.path.dirname(__file__))

NW, BD = 8, 8   # LANE_NW, LANE_BD (fpf_internal.h)


def _plan(f):
    L = _lib.load()
    dl = np.asfortranarray(f.Dl, dtype=np.float64)
    Z = np.asarray(f.Z, dtype=np.complex128)
    zb = np.zeros(max(2 * Z.size, 2))
    zb[0:2 * Z.size:2] = Z.real.ravel(order="F")
    zb[1:2 * Z.size:2] = Z.imag.ravel(order="F")
    o = _lib.FpfOpts()
    L.fpf_opts_default(C.byref(o))
    out = (C.c_int * 8)()
    slots = (C.c_int * (NW * 16 * 4))()
    blk = (C.c_int * (4096 * (1 + 2 * BD)))()
    rc = L.fpf_feeder_lane_plan(dl.ctypes.data_as(_lib._dp), dl.shape[0], dl.shape[1], zb.ctypes.data_as(_lib._dp),
                                Z.shape[0], Z.shape[1], C.byref(o), out, slots, len(slots), blk, len(blk))
    assert rc == 0
    p = dict(zip(["ok", "ns", "nw", "lds", "nE", "nG", "nblk", "n"], list(out)))
    if p["ok"]:
        # ([waves][4][slots] on the device: one scalar load per field)
        p["slots"] = np.array(slots[:NW * p["ns"] * 4], dtype=np.int64).reshape(NW, 4, p["ns"]).transpose(0, 2, 1)
        p["blk"] = np.array(blk[:p["nblk"] * (1 + 2 * BD)], dtype=np.int64).reshape(p["nblk"], 1 + 2 * BD)
    return p


def test_123bus_plan():
    f = F.synthetic_feeder(123, 123)
    p = _plan(f)
    assert p["ok"] == 1 and p["ns"] == 16 and p["nw"] == 8 and p["n"] == 122
    # 122 positions over 8 waves: 16, 16, 15, ... (2 x 16 + 6 x 15); the published
    # entries of DESIGN 6.6: 12 subtree ends, 22 taps / first - 1 positions
    assert (p["nE"], p["nG"]) == (12, 22)
    assert p["lds"] <= 159 * 1024
    nodes = p["slots"][:, :, 1]
    real = nodes[nodes >= 0]
    assert sorted(real.tolist()) == list(range(1, 123))
    for w in range(NW):
        k = (nodes[w] >= 0).sum()
        assert k == (16 if w < 2 else 15)
        assert (nodes[w, :k] >= 0).all() and (nodes[w, k:] < 0).all()   # dummies end the run
        assert p["slots"][w, 0, 3] & (1 << 30)   # every wave resolves its first block offset


@pytest.mark.parametrize("n,ns", [(9, 4), (30, 4), (34, 8), (60, 8), (97, 12), (98, 16), (129, 16), (130, 0)])
def test_plan_sizes(n, ns):
    f = F.demo_feeder() if n == 9 else F.synthetic_feeder(n, n)
    p = _plan(f)
    assert p["ok"] == (1 if ns else 0)
    if ns:
        assert p["ns"] == ns and NW * p["ns"] >= p["n"]


def test_declines():
    from test_gpu_wave import _zeroed_feeder, nested_feeder
    assert _plan(_zeroed_feeder())["ok"] == 0              # zeroed phases
    assert _plan(nested_feeder(depth=9))["ok"] == 0         # block nesting 10 > LANE_BD
    assert _plan(nested_feeder(depth=6, extra=10))["ok"] == 1


def _temp(f, bkva=1000.0, bkv=12.47):
    """TEMP = lng Z(code)/Zb of every Dl row (DPF_return7.cpp:54-80, 163-178)."""
    Zb = 1000 * bkv ** 2 / bkva
    T = {}
    for m in range(f.Dl.shape[0]):
        if f.Dl[m, 0] == 0:
            continue
        c = int(f.Dl[m, 3]) - 1
        T[m] = f.Dl[m, 4] * (f.Z[3 * c:3 * c + 3, :] / Zb)
    return T


def lane_emulate(f, p, pq, eps=1e-4, mxitr=20, bkva=1000.0, vo=1.015):
    """The lane kernel's sweep in numpy on the plan's tables, all scenarios at
    once (the same association of sums as the kernel, complex arithmetic)."""
    ns, sl, bt = p["ns"], p["slots"], p["blk"]
    B = pq.shape[2]
    s3 = bkva / 3
    v0 = np.array([vo, vo * complex(-0.5, -0.5 * np.sqrt(3)), vo * complex(-0.5, 0.5 * np.sqrt(3))])
    T = _temp(f, bkva)
    zero = max(p["nE"], p["nG"])
    x = np.tile(v0[None, None, :, None], (NW, ns, 1, B)).astype(complex)
    ibo = np.zeros((3, B), complex)
    done = np.zeros(B, bool)
    iters = np.zeros(B, int)
    nn = int((f.Dl[:, 0] != 0).sum()) + 1
    V = np.zeros((3, nn, B), complex)
    V[:, 0, :] = v0[:, None]
    loss = np.zeros(B)
    for it in range(mxitr):
        EG = np.zeros((zero + 1, 3, B), complex)
        wt = np.zeros((NW, 3, B), complex)
        for w in range(NW):
            run = np.zeros((3, B), complex)
            for i in range(ns):
                row, node = sl[w, i, 0], sl[w, i, 1]
                S = pq[0:6:2, row, :] + 1j * pq[1:6:2, row, :]
                il = np.conj(S / x[w, i]) / s3 if node >= 0 else np.zeros((3, B), complex)
                run = run + il
                x[w, i] = run
            wt[w] = run
        carry = np.cumsum(np.concatenate([np.zeros((1, 3, B)), wt[:-1]]), axis=0)
        tot = wt.sum(axis=0)
        err = np.abs(tot - ibo).max(axis=0)
        ibo = tot
        conv = err < eps
        fin = ~done & (conv | (it == mxitr - 1))
        for w in range(NW):
            x[w] += carry[w][None]
            for i in range(ns):
                pe = ((sl[w, i, 2] >> 1) & 0x7fff) - 1
                if pe >= 0:
                    EG[pe] = x[w, i]
        lp = np.zeros(B)
        for w in range(NW):
            for i in range(ns - 1, -1, -1):
                el = EG[(sl[w, i, 2] >> 16) & 0xffff]
                ib = el - (x[w, i - 1] if i > 0 else carry[w])
                row, node = sl[w, i, 0], sl[w, i, 1]
                drop = np.einsum("lb,la->ab", ib, T[row]) if node >= 0 else np.zeros((3, B), complex)
                lp += np.real(drop * np.conj(ib)).sum(axis=0)
                x[w, i] = drop
            x[w] = np.cumsum(x[w], axis=0)
        wg = np.array([x[w, ns - 1] for w in range(NW)])
        carryg = np.cumsum(np.concatenate([np.zeros((1, 3, B)), wg[:-1]]), axis=0)
        EG = np.zeros((zero + 1, 3, B), complex)
        for w in range(NW):
            for i in range(ns):
                pg = (sl[w, i, 3] & 0xffff) - 1
                if pg >= 0:
                    EG[pg] = carryg[w] + x[w, i]
        for w in range(NW):
            cb = None
            for i in range(ns):
                gi = sl[w, i, 3]
                if gi & (1 << 30):
                    b = (gi >> 16) & 0x3fff
                    cb = v0[:, None] - carryg[w]
                    for j in range(bt[b, 0]):
                        cb = cb + EG[bt[b, 2 + 2 * j]] - EG[bt[b, 1 + 2 * j]]
                x[w, i] = cb - x[w, i]
                node = sl[w, i, 1]
                if node >= 0:
                    V[:, node, fin] = x[w, i][:, fin]
        loss[fin] = s3 * lp[fin]
        iters[fin] = it + 1
        done |= fin
        if done.all():
            break
    return {"V": V, "iters": iters, "loss": loss}


@pytest.mark.parametrize("name", ["123", "60", "30", "demo", "nested"])
def test_lane_algebra_matches_oracle(name):
    from oracle import oracle as O
    from test_gpu_wave import nested_feeder
    f = {"123": lambda: F.synthetic_feeder(123, 123), "60": lambda: F.synthetic_feeder(60, 60),
         "30": lambda: F.synthetic_feeder(30, 30), "demo": F.demo_feeder,
         "nested": lambda: nested_feeder(depth=6, extra=10)}[name]()
    p = _plan(f)
    assert p["ok"] == 1
    pq = F.scenario_loads(f, np.arange(24))
    r = lane_emulate(f, p, pq)
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=4)
    assert (r["iters"] == c["iters"]).all()
    Vc = c["V_re"] + 1j * c["V_im"]
    assert np.max(np.abs(r["V"] - Vc) / np.abs(Vc)) <= 1e-12
    np.testing.assert_allclose(r["loss"], c["loss"], rtol=1e-9)


# seeded synthetic feeders of every slot count (NS 4 / 8 / 12 / 16), lateral
# counts and lengths varied: the plan and its algebra against the oracle
FUZZ = [(20, 7, None), (33, 11, 2), (47, 3, 9), (77, 21, 4), (101, 5, 20), (113, 17, 1), (128, 9, 12)]


@pytest.mark.parametrize("n,seed,lat", FUZZ)
def test_lane_algebra_random_feeders(n, seed, lat):
    from oracle import oracle as O
    f = F.synthetic_feeder(n, seed, n_laterals=lat)
    p = _plan(f)
    assert p["ok"] == 1, (n, seed, lat)
    pq = F.scenario_loads(f, np.arange(12), seed=seed)
    r = lane_emulate(f, p, pq)
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=4)
    assert (r["iters"] == c["iters"]).all()
    Vc = c["V_re"] + 1j * c["V_im"]
    assert np.max(np.abs(r["V"] - Vc) / np.abs(Vc)) <= 1e-12

