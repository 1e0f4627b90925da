"""GPU tests of the lane kernel (fpf_lane.hip: one lane per scenario, the
feeder's positions dealt to the eight waves of a workgroup) against the oracle
at the north-star bar -- V within 1e-10 relative, identical iteration counts and
status (Broker/src/vvc/DPF_return7.cpp:104-217), loss / Vmin / Vmax
(VoltVarCtrl.cpp:1152-1161, 1201-1207) -- and against the wave kernel it
replaces for large light-output batches.  FPF_LANE=1 routes every eligible
launch to it; fpf_lane_launches() counts the launches that ran it."""
import ctypes as C

import numpy as np
import pytest

from freedm_amd import feeder as F

pytestmark = pytest.mark.gpu


def _launches():
    from freedm_amd import _lib
    L = _lib.load()
    L.fpf_lane_launches.restype = C.c_int
    return int(L.fpf_lane_launches())


def _dma_launches():
    from freedm_amd import _lib
    return int(_lib.load().fpf_lane_dma_launches())


def _vrel(a, b):
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300)))


def _solve_light(pf, pq, agg=False):
    import torch
    dev = torch.device("cuda:0")
    B = pq.shape[2]
    out = {"v_re": torch.zeros((3, pf.nn, B), dtype=torch.float64, device=dev),
           "v_im": torch.zeros((3, pf.nn, B), dtype=torch.float64, device=dev),
           "iters": torch.zeros(B, dtype=torch.int32, device=dev), "status": torch.zeros(B, dtype=torch.int8, device=dev),
           "loss": torch.zeros(B, dtype=torch.float64, device=dev), "vmin": torch.zeros(B, dtype=torch.float64, device=dev),
           "vmax": torch.zeros(B, dtype=torch.float64, device=dev),
           "errmx": torch.zeros(B, dtype=torch.float64, device=dev), "guard": torch.zeros(B, dtype=torch.int8, device=dev)}
    a = torch.zeros(8, dtype=torch.float64, device=dev) if agg else None
    pf.solve_device(torch.from_numpy(np.ascontiguousarray(pq)).to(dev), out, agg=a)
    torch.cuda.synchronize()
    r = {k: v.cpu().numpy() for k, v in out.items()}
    r["V"] = r["v_re"] + 1j * r["v_im"]
    if agg:
        r["agg"] = a.cpu().numpy()
    return r


def _check_oracle(f, pq, r):
    from oracle import oracle as O
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    assert (r["iters"] == c["iters"]).all(), (r["iters"], c["iters"])
    assert (r["status"] == c["status"]).all()
    conv = c["status"] == 0
    assert conv.any()
    assert _vrel(r["V"][..., conv], (c["V_re"] + 1j * c["V_im"])[..., conv]) <= 1e-10
    np.testing.assert_allclose(r["loss"][conv], c["loss"][conv], rtol=1e-8, atol=1e-9)
    np.testing.assert_allclose(r["vmin"][conv], c["vmin"][conv], rtol=1e-10)
    np.testing.assert_allclose(r["vmax"][conv], c["vmax"][conv], rtol=1e-10)
    np.testing.assert_allclose(r["errmx"], c["errmx"], rtol=1e-8)
    return c


def _feeder(name):
    if name == "demo":
        return F.demo_feeder()
    return F.synthetic_feeder(int(name), int(name))


# 123-bus: 16 slots per wave (6 dummies); 60: 8; 30 and the 9-row demo: 4 (one real
# slot per wave, the rest dummies)
@pytest.mark.parametrize("name,B", [("123", 1), ("123", 37), ("123", 64), ("123", 4133), ("60", 300),
                                    ("30", 129), ("demo", 65)])
def test_lane_matches_oracle(name, B, monkeypatch):
    from freedm_amd import PowerFlow
    monkeypatch.setenv("FPF_LANE", "1")
    f = _feeder(name)
    pq = F.scenario_loads(f, np.arange(500, 500 + B))
    pf = PowerFlow(f)
    n0, d0 = _launches(), _dma_launches()
    r = _solve_light(pf, pq)
    assert _launches() == n0 + 1, "the lane kernel did not run"
    assert _dma_launches() == d0   # (the LDS-DMA ring only on request, FPF_LANE_DMA=1)
    _check_oracle(f, pq, r)
    assert not r["guard"].any()


def test_lane_matches_wave_kernel(monkeypatch):
    """The same hosting batch on the lane and the wave kernel: identical iteration
    counts and status, V within 1e-12, the scalars within their rounding."""
    from freedm_amd import PowerFlow
    f = F.synthetic_feeder(123, 123)
    pq = F.hosting_loads(f, np.arange(8192), seed=2 ** 20)
    pf = PowerFlow(f)
    monkeypatch.setenv("FPF_LANE", "0")
    w = _solve_light(pf, pq, agg=True)
    monkeypatch.setenv("FPF_LANE", "1")
    n0 = _launches()
    lr = _solve_light(pf, pq, agg=True)
    assert _launches() == n0 + 1
    np.testing.assert_array_equal(lr["iters"], w["iters"])
    np.testing.assert_array_equal(lr["status"], w["status"])
    assert _vrel(lr["V"], w["V"]) <= 1e-12
    np.testing.assert_allclose(lr["loss"], w["loss"], rtol=1e-9)
    np.testing.assert_allclose(lr["vmin"], w["vmin"], rtol=1e-13)
    np.testing.assert_allclose(lr["vmax"], w["vmax"], rtol=1e-13)
    # the fused aggregate (tile partials of 64 scenarios, folded in order)
    np.testing.assert_array_equal(lr["agg"][3:], w["agg"][3:])
    assert lr["agg"][0] == pytest.approx(w["agg"][0], rel=1e-12)
    assert lr["agg"][1] == pytest.approx(w["agg"][1], rel=1e-13)
    assert lr["agg"][2] == pytest.approx(w["agg"][2], rel=1e-13)
    assert lr["agg"][7] == pq.shape[2]


def test_lane_dma_ring_equals_register_loads(monkeypatch):
    """The same even batch with the loads through the LDS-DMA ring (FPF_LANE_DMA=1)
    and through registers: the same arithmetic on the same values, so every output
    is bit-identical; ragged last workgroup (B % 64 != 0); an odd batch keeps the
    register loads (a lane's 16-byte piece is two scenarios)."""
    from freedm_amd import PowerFlow
    monkeypatch.setenv("FPF_LANE", "1")
    monkeypatch.setenv("FPF_LANE_DMA", "1")
    f = F.synthetic_feeder(123, 123)
    pq = F.hosting_loads(f, np.arange(3000), seed=77)
    pf = PowerFlow(f)
    d0 = _dma_launches()
    a = _solve_light(pf, pq, agg=True)
    assert _dma_launches() == d0 + 1
    _solve_light(pf, np.ascontiguousarray(pq[:, :, :2999]))
    assert _dma_launches() == d0 + 1
    monkeypatch.setenv("FPF_LANE_DMA", "0")
    b = _solve_light(pf, pq, agg=True)
    assert _dma_launches() == d0 + 1
    for k in ("v_re", "v_im", "iters", "status", "loss", "vmin", "vmax", "errmx", "agg"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_lane_nonconverged_and_mxitr(monkeypatch):
    """Heavy loads that do not converge in mxitr sweeps: status 1 and iters =
    mxitr, as the oracle (the reference throws there, DPF_return7.cpp:242)."""
    from freedm_amd import PowerFlow
    monkeypatch.setenv("FPF_LANE", "1")
    f = F.synthetic_feeder(123, 123)
    pq = F.scenario_loads(f, np.arange(128))
    pq[:, :, ::3] *= 40.0   # every third scenario far past the loadability
    pf = PowerFlow(f)
    r = _solve_light(pf, pq)
    from oracle import oracle as O
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    assert (c["status"] != 0).any() and (c["status"] == 0).any()
    np.testing.assert_array_equal(r["iters"], c["iters"])
    np.testing.assert_array_equal(r["status"], c["status"])
    conv = c["status"] == 0
    assert _vrel(r["V"][..., conv], (c["V_re"] + 1j * c["V_im"])[..., conv]) <= 1e-10


def test_lane_near_eps_guard(monkeypatch):
    """Scenarios whose deciding errmx sits on eps (tests/near_eps.py): the lane
    kernel sums Ib(0) in yet another order; the guard flags them and the exact
    re-solve makes the sweep counts the oracle's, with and without an aggregate."""
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    from near_eps import near_eps_batch
    monkeypatch.setenv("FPF_LANE", "1")
    f = F.synthetic_feeder(123, 123)
    base = F.scenario_loads(f, np.arange(40))
    a, _ = near_eps_batch(O, f, base, 6, 0.05, 1.0)
    b, _ = near_eps_batch(O, f, base, 6, 1.0, 3.0)
    pq = np.ascontiguousarray(np.concatenate([a, b], axis=2))
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    pf = PowerFlow(f)
    for agg in (False, True):
        n0 = _launches()
        r = _solve_light(pf, pq, agg=agg)
        assert _launches() == n0 + 1
        assert (r["iters"] == c["iters"]).all(), (r["iters"], c["iters"])
        assert (r["status"] == c["status"]).all()
        assert (r["guard"] == 1).all(), r["guard"]
        np.testing.assert_array_equal(r["v_re"], c["V_re"])
        np.testing.assert_array_equal(r["v_im"], c["V_im"])


def test_lane_declines_and_wave_runs(monkeypatch):
    """Feeders outside the lane plan (zeroed phases; block nesting deeper than
    LANE_BD) and full outputs / scenario-major batches keep the wave kernel."""
    from freedm_amd import PowerFlow
    from test_gpu_wave import _zeroed_feeder, nested_feeder
    monkeypatch.setenv("FPF_LANE", "1")
    for f in (_zeroed_feeder(), nested_feeder(depth=9)):
        pq = F.scenario_loads(f, np.arange(70))
        n0 = _launches()
        r = _solve_light(PowerFlow(f), pq)
        assert _launches() == n0
        _check_oracle(f, pq, r)
    f = F.synthetic_feeder(123, 123)
    pq = F.scenario_loads(f, np.arange(70))
    n0 = _launches()
    PowerFlow(f).solve(pq)   # full outputs (Vpolar, PQb, PQL)
    r = _solve_light(PowerFlow(f), pq)
    assert _launches() == n0 + 1   # (light outputs with both V planes: the lane kernel)
    n0 = _launches()
    import torch
    one = {"v_re": torch.zeros((3, PowerFlow(f).nn, 70), dtype=torch.float64, device="cuda:0")}
    PowerFlow(f).solve_device(torch.from_numpy(pq).to("cuda:0"), one)   # one V plane: the wave kernel
    torch.cuda.synchronize()
    np.testing.assert_allclose(one["v_re"].cpu().numpy(), r["v_re"], rtol=1e-12, atol=1e-14)
    PowerFlow(f, layout=1).solve(np.ascontiguousarray(pq.transpose(2, 0, 1)), full=False)
    assert _launches() == n0


def test_lane_two_streams(monkeypatch):
    """Lane launches on two streams with caller-owned outputs overlap freely and
    give the same results as one at a time."""
    import torch
    from freedm_amd import PowerFlow
    monkeypatch.setenv("FPF_LANE", "1")
    f = F.synthetic_feeder(123, 123)
    pf = PowerFlow(f)
    xs = [F.scenario_loads(f, np.arange(k * 640, k * 640 + 640)) for k in range(2)]
    ref = [_solve_light(pf, x) for x in xs]
    dev = torch.device("cuda:0")
    d = [torch.from_numpy(x).to(dev) for x in xs]
    outs = [{"v_re": torch.zeros((3, pf.nn, 640), dtype=torch.float64, device=dev),
             "v_im": torch.zeros((3, pf.nn, 640), dtype=torch.float64, device=dev),
             "iters": torch.zeros(640, dtype=torch.int32, device=dev),
             "status": torch.zeros(640, dtype=torch.int8, device=dev),
             "loss": torch.zeros(640, dtype=torch.float64, device=dev),
             "vmin": torch.zeros(640, dtype=torch.float64, device=dev),
             "vmax": torch.zeros(640, dtype=torch.float64, device=dev)} for _ in range(2)]
    s = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    n0 = _launches()
    for _ in range(3):
        for k in range(2):
            pf.solve_device(d[k], outs[k], stream=s[k])
    torch.cuda.synchronize()
    assert _launches() == n0 + 6
    for k in range(2):
        np.testing.assert_array_equal(outs[k]["v_re"].cpu().numpy(), ref[k]["v_re"])
        np.testing.assert_array_equal(outs[k]["v_im"].cpu().numpy(), ref[k]["v_im"])
        np.testing.assert_array_equal(outs[k]["iters"].cpu().numpy(), ref[k]["iters"])
        np.testing.assert_array_equal(outs[k]["loss"].cpu().numpy(), ref[k]["loss"])


@pytest.mark.parametrize("n,seed,lat", [(20, 7, None), (47, 3, 9), (77, 21, 4), (101, 5, 20), (128, 9, 12)])
def test_lane_random_feeders(n, seed, lat, monkeypatch):
    """Seeded synthetic feeders of every slot count (tests/test_lane_plan.py: FUZZ)
    on the lane kernel against the oracle at the north-star bar."""
    from freedm_amd import PowerFlow
    monkeypatch.setenv("FPF_LANE", "1")
    f = F.synthetic_feeder(n, seed, n_laterals=lat)
    pq = F.scenario_loads(f, np.arange(130), seed=seed)
    pf = PowerFlow(f)
    n0 = _launches()
    r = _solve_light(pf, pq)
    assert _launches() == n0 + 1
    _check_oracle(f, pq, r)


def test_lane_nested_blocks(monkeypatch):
    """Block chains six deep with ten one-node laterals (the plan's block table,
    tests/test_lane_plan.py: the algebra on CPU) on the GPU."""
    from freedm_amd import PowerFlow
    from test_gpu_wave import nested_feeder
    monkeypatch.setenv("FPF_LANE", "1")
    f = nested_feeder(depth=6, extra=10)
    pq = F.scenario_loads(f, np.arange(200))
    n0 = _launches()
    r = _solve_light(PowerFlow(f), pq)
    assert _launches() == n0 + 1
    _check_oracle(f, pq, r)

