"""GPU tests of the wave kernel's structural paths (fpf_wave.hip) against the
oracle at the north-star bar (V within 1e-10 relative, identical iteration
counts): ragged batches, deeply nested laterals with more blocks than a
segment has lanes (the LDS block-chain path), a lateral whose first branch
zeroes phases its children carry (V = A(m) - A(k) below a zeroed ancestor),
every geometry (scenarios per wave x slots per lane), and the light variant
(V and VVC scalars only) against the full one."""
import os

import numpy as np
import pytest

from freedm_amd import feeder as F

pytestmark = pytest.mark.gpu


def _vrel(a, b):
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300)))


def _check(f, pq, **kw):
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    pf = PowerFlow(f, kernel="wave", **kw)
    r = pf.solve(pq)
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    assert (r["iters"] == c["iters"]).all() and (r["status"] == c["status"]).all()
    conv = c["status"] == 0
    assert conv.any()
    assert _vrel((r["V_re"] + 1j * r["V_im"])[..., conv], (c["V_re"] + 1j * c["V_im"])[..., conv]) <= 1e-10
    np.testing.assert_allclose(r["loss"][conv], c["loss"][conv], rtol=1e-8, atol=1e-9)
    np.testing.assert_allclose(r["vmin"][conv], c["vmin"][conv], rtol=1e-10)
    np.testing.assert_allclose(r["vmax"][conv], c["vmax"][conv], rtol=1e-10)
    return pf, r


def nested_feeder(main_len=12, depth=9, lat_len=3, extra=30, seed=5):
    """A radial Dl table with a chain of `depth` laterals each tapping the previous
    lateral's last node (block-chain depth > 4) and `extra` one-node laterals
    (more blocks than the 32 lanes of a segment)."""
    rng = np.random.default_rng(seed)
    rows = [(0, 1, 2)]   # substation transformer, code 2
    node = 1
    for _ in range(main_len):
        rows.append((node, node + 1, 1))
        node += 1
    tap = 3
    for _ in range(depth):
        rows.append(None)
        prev = tap
        for _ in range(lat_len):
            rows.append((prev, node + 1, 1))
            prev = node + 1
            node += 1
        tap = prev
    for _ in range(extra):
        rows.append(None)
        rows.append((int(rng.integers(1, node + 1)), node + 1, 1))
        node += 1
    Dl = np.zeros((len(rows), F.N_COLS))
    ln = 0
    for i, r in enumerate(rows):
        if r is None:
            continue
        ln += 1
        Dl[i, 0:5] = (ln, r[0], r[1], r[2], rng.uniform(0.02, 0.1))
        Dl[i, 5] = 1
        if i > 0:
            p = rng.uniform(0.0, 3.0, 3)
            Dl[i, 6:12:2] = np.round(p, 3)
            Dl[i, 7:12:2] = np.round(0.3 * p, 3)
    return F.Feeder(Dl, F.demo_feeder().Z, name="nested")


@pytest.mark.parametrize("B", [1, 15, 16, 17, 33])
def test_ragged_batches(B):
    f = F.synthetic_feeder(123, 123)
    _check(f, F.scenario_loads(f, np.arange(1000, 1000 + B)))


def test_deep_nesting_and_many_blocks():
    f = nested_feeder()
    assert int((f.Dl[:, 0] != 0).sum()) <= 128
    _check(f, F.scenario_loads(f, np.arange(64)))


def test_zeroed_phase_with_carrying_children():
    f = F.demo_feeder()
    Z = np.vstack([f.Z, np.diag([0, 2.0 + 6.0j, 0])])
    Dl = f.Dl.copy()
    Dl[6, 3] = 3            # the lateral's first branch carries phase B only
    Dl[7:9, [6, 7, 10, 11]] = 0   # no A/C load below it: V there is -drop (mutual coupling), small
    g = F.Feeder(Dl, Z, name="demo-rel")
    _check(g, F.scenario_loads(g, np.arange(24)))


@pytest.mark.parametrize("n_nodes,geom", [(9, "4,1"), (30, "4,2"), (60, "2,2"), (123, "2,4"), (123, "1,4"),
                                          (123, "1,2"), (200, "1,4")])
def test_every_geometry(n_nodes, geom, monkeypatch):
    monkeypatch.setenv("FPF_WAVE_GEOM", geom)
    f = F.synthetic_feeder(n_nodes, n_nodes) if n_nodes > 9 else F.demo_feeder()
    pf, _ = _check(f, F.scenario_loads(f, np.arange(40)))
    spw = int(geom.split(",")[0])
    if int((f.Dl[:, 0] != 0).sum()) <= (64 // spw) * int(geom.split(",")[1]):
        assert pf.info["tile"] in (4 * spw, 8 * spw, 16 * spw)


def test_light_outputs_match_full():
    import torch
    from freedm_amd import PowerFlow
    f = F.synthetic_feeder(123, 123)
    pq = F.scenario_loads(f, np.arange(300))
    pf = PowerFlow(f, kernel="wave")
    full = pf.solve(pq)
    dev = torch.device("cuda:0")
    B = pq.shape[2]
    out = {"v_re": torch.zeros((3, pf.nn, B), dtype=torch.float64, device=dev),
           "v_im": torch.zeros((3, pf.nn, B), dtype=torch.float64, device=dev),
           "iters": torch.zeros(B, dtype=torch.int32, device=dev), "status": torch.zeros(B, dtype=torch.int8, device=dev),
           "loss": torch.zeros(B, dtype=torch.float64, device=dev), "vmin": torch.zeros(B, dtype=torch.float64, device=dev),
           "vmax": torch.zeros(B, dtype=torch.float64, device=dev)}
    pf.solve_device(torch.from_numpy(pq).to(dev), out)
    torch.cuda.synchronize()
    for k, h in (("v_re", "V_re"), ("v_im", "V_im"), ("iters", "iters"), ("loss", "loss"), ("vmin", "vmin"),
                 ("vmax", "vmax")):
        np.testing.assert_array_equal(out[k].cpu().numpy(), full[h], err_msg=k)


def _zeroed_feeder():
    f = F.demo_feeder()
    Z = np.vstack([f.Z, np.diag([0, 2.0 + 6.0j, 0])])
    Dl = f.Dl.copy()
    Dl[6, 3] = 3
    Dl[7:9, [6, 7, 10, 11]] = 0
    return F.Feeder(Dl, Z, name="demo-rel")


@pytest.mark.parametrize("which", ["123", "123-1,4", "30", "nested", "zeroed"])
def test_specialised_build_matches_static(which, monkeypatch):
    """fpf_opts.specialize with FPF_WAVE_RTC=2048: a light-output wave launch of
    >= 2048 scenarios runs the per-plan hipRTC build (fpf_rtc.cpp:
    wave_rtc_function) -- the same source with the plan's values as constants,
    so every output is the static kernel's bit for bit; full outputs (and zeroed
    phases) run the static kernel either way; both are the oracle's at the
    north-star bar."""
    import ctypes as C
    import torch
    from freedm_amd import PowerFlow, _lib
    monkeypatch.setenv("FPF_WAVE_RTC", "2048")
    if which == "123-1,4":
        monkeypatch.setenv("FPF_WAVE_GEOM", "1,4")
    f = {"123": lambda: F.synthetic_feeder(123, 123), "123-1,4": lambda: F.synthetic_feeder(123, 123),
         "30": lambda: F.synthetic_feeder(30, 30), "nested": nested_feeder, "zeroed": _zeroed_feeder}[which]()
    B = 2304
    pq = F.scenario_loads(f, np.arange(B))
    L = _lib.load()
    L.fpf_wave_rtc_builds.restype = C.c_int
    n0 = L.fpf_wave_rtc_builds()
    spec = PowerFlow(f, kernel="wave")
    stat = PowerFlow(f, kernel="wave", specialize=False)
    a, b = spec.solve(pq), stat.solve(pq)   # (full outputs: the static kernel both)
    for k in a:
        np.testing.assert_array_equal(np.asarray(a[k]), np.asarray(b[k]), err_msg=k)
    dev = torch.device("cuda:0")
    res = []
    for pf in (spec, stat):
        out = {"v_re": torch.zeros((3, pf.nn, B), dtype=torch.float64, device=dev),
               "v_im": torch.zeros((3, pf.nn, B), dtype=torch.float64, device=dev),
               "iters": torch.zeros(B, dtype=torch.int32, device=dev),
               "status": torch.zeros(B, dtype=torch.int8, device=dev),
               "loss": torch.zeros(B, dtype=torch.float64, device=dev),
               "vmin": torch.zeros(B, dtype=torch.float64, device=dev),
               "vmax": torch.zeros(B, dtype=torch.float64, device=dev)}
        pf.solve_device(torch.from_numpy(pq).to(dev), out)
        torch.cuda.synchronize()
        res.append({k: v.cpu().numpy() for k, v in out.items()})
    for k in res[0]:
        np.testing.assert_array_equal(res[0][k], res[1][k], err_msg="light " + k)
    # the light variant of a feeder without zeroed phases ran the hipRTC build
    # (here or in an earlier test of the same plan)
    n1 = L.fpf_wave_rtc_builds()
    assert n1 >= n0 and (n1 >= 1 or which == "zeroed")
    # and the oracle, on a slice
    _check(f, pq[:, :, :64])
