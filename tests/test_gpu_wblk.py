"""The wave-block kernel (fpf_wblk.hip; fast mode on feeders of 257..2048
branches, one scenario per workgroup of 2, 4 or 8 wavefronts) against the
oracle and against the exact generic kernel on the same inputs.

Bar (north_star, as for the per-wavefront wave kernel in test_gpu_parity.py):
V within 1e-10 relative and identical iteration counts and status on every
scenario; PQb / PQL / Vpolar at 1e-9 (angles 1e-8 deg), loss 1e-8, Vmin/Vmax
1e-10.  The reference: DPF_return7.cpp:8-263 and the VVC reductions
(VoltVarCtrl.cpp:1152-1161, 1201-1207), restated by oracle/ref_dpf.c.
"""
import os

import numpy as np
import pytest

from freedm_amd import feeder as F

pytestmark = pytest.mark.gpu


def _vrel(a_re, a_im, b_re, b_im):
    a = a_re + 1j * a_im
    b = b_re + 1j * b_im
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300)))


def _close(a, b, rtol):
    scale = max(float(np.max(np.abs(b))), 1e-300)
    assert float(np.max(np.abs(a - b))) <= rtol * scale, (float(np.max(np.abs(a - b))), scale)


def _check_full(r, c):
    assert (r["iters"] == c["iters"]).all() and (r["status"] == c["status"]).all()
    conv = c["status"] == 0
    assert _vrel(r["V_re"][..., conv], r["V_im"][..., conv], c["V_re"][..., conv], c["V_im"][..., conv]) <= 1e-10
    _close(r["loss"][conv], c["loss"][conv], 1e-8)
    np.testing.assert_allclose(r["vmin"][conv], c["vmin"][conv], rtol=1e-10)
    np.testing.assert_allclose(r["vmax"][conv], c["vmax"][conv], rtol=1e-10)
    _close(r["PQb"][..., conv], c["PQb"][..., conv], 1e-9)
    _close(r["PQL"][..., conv], c["PQL"][..., conv], 1e-9)
    np.testing.assert_allclose(r["Vpolar"][0::2][..., conv], c["Vpolar"][0::2][..., conv], rtol=1e-10, atol=0)
    np.testing.assert_allclose(r["Vpolar"][1::2][..., conv], c["Vpolar"][1::2][..., conv], rtol=0, atol=1e-8)


@pytest.mark.parametrize("n,wps", [(300, 2), (700, 4), (1100, 8), (2048, 8)])
def test_wblk_matches_oracle(n, wps):
    """Every geometry (2, 4, 8 wavefronts per scenario), full outputs, against
    the oracle scenario by scenario."""
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    f = F.synthetic_feeder(n, n)
    pq = F.scenario_loads(f, np.arange(48))
    pf = PowerFlow(f)
    assert pf.kernel == "wave" and pf.info["tile"] == 1
    r = pf.solve(pq)
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    assert (c["status"] == 0).all()
    _check_full(r, c)


def test_wblk_nonconvergent_and_mixed_sweeps():
    """Loads scaled 0.05x .. 60x: scenarios converge after different numbers of
    sweeps and the heaviest never converge (status 1 after 20 sweeps, where the
    reference throws, DPF_return7.cpp:242) -- iteration counts and status
    identical to the oracle, V of the converged ones at the bar."""
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    f = F.synthetic_feeder(700, 700)
    pq = F.scenario_loads(f, np.arange(40))
    scale = np.geomspace(0.05, 60.0, 40)
    pq = np.ascontiguousarray(pq * scale[None, None, :])
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    assert (c["status"] == 1).any() and (c["status"] == 0).any() and len(set(c["iters"][c["status"] == 0])) >= 3
    r = PowerFlow(f).solve(pq)
    _check_full(r, c)


def _masked_feeder(n=700, seed=700, restart=False):
    """Synthetic feeder with zeroed phases: a phase-B-only line code on every row
    of two laterals (phases A and C zeroed there, DPF_return7.cpp:180-192); with
    restart, on the first row only of the second (its three-phase rows below
    restart from a zeroed ancestor -- not a physical feeder, but a table the
    reference solves); the loads of phases A and C removed on both laterals."""
    f = F.synthetic_feeder(n, seed)
    Dl = f.Dl.copy()
    Z = np.vstack([f.Z, np.diag([0, 0.3 + 0.8j, 0])])
    code = Z.shape[0] // 3
    seps = np.flatnonzero(Dl[:, 0] == 0)

    def block(i):
        return seps[i] + 1, (seps[i + 1] if i + 1 < len(seps) else Dl.shape[0])
    a, b = block(3)
    Dl[a:b, 3] = code
    Dl[a:b, [6, 7, 10, 11]] = 0
    a, b = block(7)
    if restart:
        Dl[a, 3] = code
    else:
        Dl[a:b, 3] = code
    Dl[a:b, [6, 7, 10, 11]] = 0
    return F.Feeder(Dl, Z, name=f"synthetic-{n}bus-zeroed-phases")


@pytest.mark.parametrize("n", [700, 2048])
def test_wblk_zeroed_phases(n):
    """Zeroed phases on the wave-block kernel (the full-output variant): V = 0
    on the zeroed phases and the -180/+180 angle pattern, the restart below a
    zeroed ancestor, the loss over PQL and the general V_abc_list extremes
    (Lnum_p + 1 < Nn), against the oracle."""
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    from test_gpu_parity import _fast_mode_outputs_match
    f = _masked_feeder(n, n)
    pq = F.scenario_loads(f, np.arange(24), pv_frac=0.0)
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    assert (c["status"] == 0).all()
    assert (c["Vpolar"][0::2] == 0).any()                      # some (node, phase) zeroed
    nn = int((f.Dl[:, 0] != 0).sum()) + 1
    assert min(O.lnum(f.Dl, f.Z)) + 1 < nn                     # V_abc_list drops rows
    pf = PowerFlow(f)
    assert pf.kernel == "wave" and pf.info["tile"] == 1
    r = pf.solve(pq)
    assert (r["iters"] == c["iters"]).all() and (r["status"] == c["status"]).all()
    assert _vrel(r["V_re"], r["V_im"], c["V_re"], c["V_im"]) <= 1e-10   # zeroed entries: exactly 0 in both
    _close(r["loss"], c["loss"], 1e-8)
    np.testing.assert_allclose(r["vmin"], c["vmin"], rtol=1e-10)
    np.testing.assert_allclose(r["vmax"], c["vmax"], rtol=1e-10)
    _fast_mode_outputs_match(r, c, c["status"] == 0)


@pytest.mark.parametrize("n", [700, 2048])
def test_wblk_restart_below_zeroed_phase(n):
    """A live phase below a zeroed ancestor m (V(k) = A(m) - A(k), the path
    restarting from 0 at m, DPF_return7.cpp:180-195; not a physical feeder but a
    table the reference solves) on the wave-block kernel: its forward scan is
    segmented at block heads, so V(k) is a difference of two small path sums
    (the unsegmented prefix sums over up to 2048 positions missed the bar there:
    3.8e-10) -- iteration counts identical, V within 1e-10 relative against the
    oracle (the margin printed), the full outputs at the fast-mode bar."""
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    from test_gpu_parity import _fast_mode_outputs_match
    f = _masked_feeder(n, n, restart=True)
    pq = F.scenario_loads(f, np.arange(16), pv_frac=0.0)
    pf = PowerFlow(f)
    assert pf.kernel == "wave" and pf.info["tile"] == 1
    r = pf.solve(pq)
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    assert (c["status"] == 0).all()
    assert (r["iters"] == c["iters"]).all() and (r["status"] == c["status"]).all()
    e = _vrel(r["V_re"], r["V_im"], c["V_re"], c["V_im"])
    print(f"restart below a zeroed phase, {n}-bus: max V rel err {e:.3e}")
    assert e <= 1e-10
    _close(r["loss"], c["loss"], 1e-8)
    np.testing.assert_allclose(r["vmin"], c["vmin"], rtol=1e-10)
    np.testing.assert_allclose(r["vmax"], c["vmax"], rtol=1e-10)
    _fast_mode_outputs_match(r, c, c["status"] == 0)


def test_config3_wblk_full_size():
    """BASELINE config 3 at its stated size on the default (fast) path: 65 536
    scenarios of the 2048-bus feeder in one launch of the wave-block kernel,
    light outputs (V + per-scenario scalars) and the fused aggregate, against
    the exact generic kernel on the same device inputs for every scenario
    (iteration counts and status identical, V 1e-10, loss 1e-8, Vmin/Vmax
    1e-10, the aggregate's counts equal) and against the oracle on a strided
    sample."""
    import torch
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    f = F.synthetic_feeder(2048, 2048)
    B, NB = 65536, 1024
    base = F.scenario_loads(f, np.arange(NB), seed=65536)
    dev = torch.device("cuda:0")
    s = np.arange(B, dtype=np.int64)
    mult = 0.9 + 0.2 * (((s * 2654435761) % 1000) / 1000.0)
    d_pq = torch.from_numpy(base).to(dev)[:, :, torch.from_numpy(s % NB).to(dev)] * torch.from_numpy(mult).to(dev)

    def run(pf):
        nn = pf.nn
        out = {"v_re": torch.empty((3, nn, B), dtype=torch.float64, device=dev),
               "v_im": torch.empty((3, nn, B), dtype=torch.float64, device=dev),
               "iters": torch.empty(B, dtype=torch.int32, device=dev),
               "status": torch.empty(B, dtype=torch.int8, device=dev),
               "loss": torch.empty(B, dtype=torch.float64, device=dev),
               "vmin": torch.empty(B, dtype=torch.float64, device=dev),
               "vmax": torch.empty(B, dtype=torch.float64, device=dev)}
        agg = torch.zeros(8, dtype=torch.float64, device=dev)
        pf.solve_device(d_pq, out, agg=agg)
        torch.cuda.synchronize()
        return out, agg.cpu().numpy()

    fast = PowerFlow(f, device=0)
    assert fast.kernel == "wave" and fast.info["tile"] == 1
    w, wa = run(fast)
    assert wa[7] == B and wa[3] + wa[4] == B
    # scenario by scenario against the oracle on a strided sample
    idx = np.arange(0, B, 1021)
    ti = torch.from_numpy(idx).to(dev)
    pq_s = np.ascontiguousarray(base[:, :, idx % NB] * mult[idx])
    c = O.dpf_batch(f.Dl, f.Z, pq_s, nthreads=8)
    assert (w["iters"][ti].cpu().numpy() == c["iters"]).all() and (w["status"][ti].cpu().numpy() == c["status"]).all()
    assert _vrel(w["v_re"][:, :, ti].cpu().numpy(), w["v_im"][:, :, ti].cpu().numpy(), c["V_re"], c["V_im"]) <= 1e-10
    np.testing.assert_allclose(w["loss"][ti].cpu().numpy(), c["loss"], rtol=1e-8)
    np.testing.assert_allclose(w["vmin"][ti].cpu().numpy(), c["vmin"], rtol=1e-10)
    np.testing.assert_allclose(w["vmax"][ti].cpu().numpy(), c["vmax"], rtol=1e-10)
    # every scenario against the exact generic kernel
    exact = PowerFlow(f, device=0, exact=1)
    assert exact.kernel == "generic"
    g, ga = run(exact)
    assert torch.equal(w["iters"], g["iters"]) and torch.equal(w["status"], g["status"])
    a = w["v_re"] + 1j * w["v_im"]
    b = g["v_re"] + 1j * g["v_im"]
    assert float(((a - b).abs() / b.abs()).max()) <= 1e-10
    del a, b
    assert float(((w["loss"] - g["loss"]).abs() / g["loss"].abs()).max()) <= 1e-8
    assert float(((w["vmin"] - g["vmin"]).abs() / g["vmin"]).max()) <= 1e-10
    assert float(((w["vmax"] - g["vmax"]).abs() / g["vmax"]).max()) <= 1e-10
    np.testing.assert_array_equal(wa[3:], ga[3:])
    np.testing.assert_allclose(wa[:3], ga[:3], rtol=1e-8)


def test_wblk_areas_equal_monolithic():
    """The multi-area solve (fpf_areas_*, per-scenario source voltages) on a
    1100-bus feeder whose root area needs the wave-block kernel: V equals the
    monolithic solve to 1e-10 (tests/test_areas.py for the 123-bus splits)."""
    from freedm_amd import AreaPowerFlow
    from oracle import oracle as O
    f = F.synthetic_feeder(1100, 1100)
    node_area = F.subtree_node_areas(f, [200, 600])
    pq = F.scenario_loads(f, np.arange(32))
    ap = AreaPowerFlow(f, node_area)
    r = ap.solve(pq, tol=1e-13, max_outer=100)
    o = O.default_opts()
    o.eps = 1e-13
    o.mxitr = 200
    c = O.dpf_batch(f.Dl, f.Z, pq, opts=o, nthreads=8)
    assert (c["status"] == 0).all() and (r["status"] == 0).all(), r["note"]
    v = r["V_re"] + 1j * r["V_im"]
    vc = c["V_re"] + 1j * c["V_im"]
    assert float(np.max(np.abs(v - vc) / np.abs(vc))) <= 1e-10
    np.testing.assert_allclose(r["loss"], c["loss"], rtol=1e-8)


def test_wblk_heavy_2048_bus():
    """The benched 2048-bus feeder (config 3) under heavier loads than the bench's:
    scale 1.7 .. 3.3 of the calibrated scenarios (SURVEY 8(d)'s Vmin ~ 0.92 and
    below: 6 .. 12 sweeps, Vmin 0.93 .. 0.81), both batch layouts, against the
    oracle: iteration counts and status identical, V within 1e-10 relative
    (the max error is printed: the margin of the prefix-sum voltages)."""
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    f = F.synthetic_feeder(2048, 2048)
    B = 48
    pq = F.scenario_loads(f, np.arange(B)) * np.geomspace(1.7, 3.3, B)[None, None, :]
    pq = np.ascontiguousarray(pq)
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    assert (c["status"] == 0).all() and c["iters"].min() <= 7 and c["iters"].max() >= 11
    assert c["vmin"].min() < 0.85
    import torch
    dev = torch.device("cuda:0")
    for layout in (0, 1):
        pf = PowerFlow(f, layout=layout)
        assert pf.kernel == "wave" and pf.info["tile"] == 1
        x = pq if layout == 0 else np.ascontiguousarray(pq.transpose(2, 0, 1))
        # the light outputs (V and the scalars: the benched variant), device buffers
        sh = (3, pf.nn, B) if layout == 0 else (B, 3, pf.nn)
        o = {"v_re": torch.empty(sh, dtype=torch.float64, device=dev),
             "v_im": torch.empty(sh, dtype=torch.float64, device=dev),
             "iters": torch.empty(B, dtype=torch.int32, device=dev),
             "status": torch.empty(B, dtype=torch.int8, device=dev),
             "loss": torch.empty(B, dtype=torch.float64, device=dev),
             "vmin": torch.empty(B, dtype=torch.float64, device=dev)}
        pf.solve_device(torch.from_numpy(x).to(dev), o)
        torch.cuda.synchronize()
        r = {k: v.cpu().numpy() for k, v in o.items()}
        vr, vi = (r["v_re"], r["v_im"]) if layout == 0 else (np.moveaxis(r["v_re"], 0, -1), np.moveaxis(r["v_im"], 0, -1))
        assert (r["iters"] == c["iters"]).all() and (r["status"] == c["status"]).all()
        e = _vrel(vr, vi, c["V_re"], c["V_im"])
        print(f"layout {layout}: max V rel err {e:.3e}, sweeps {c['iters'].min()}..{c['iters'].max()}")
        assert e <= 1e-10
        np.testing.assert_allclose(r["vmin"], c["vmin"], rtol=1e-10)
        np.testing.assert_allclose(r["loss"], c["loss"], rtol=1e-8)
        pf.close()


@pytest.mark.parametrize("n", [300, 1100])
def test_wblk_specialised_build_matches_static(n, monkeypatch):
    """fpf_opts.specialize with FPF_WAVE_RTC=2048: a light-output wave-block
    launch of >= 2048 scenarios runs the per-plan hipRTC build (fpf_rtc.cpp:
    wave_rtc_function, fpf_wblk_body.h under FPF_WSPEC) -- every output bit for
    bit the static kernel's; the oracle on a slice."""
    import ctypes as C
    import torch
    from freedm_amd import PowerFlow, _lib
    from oracle import oracle as O
    monkeypatch.setenv("FPF_WAVE_RTC", "2048")
    f = F.synthetic_feeder(n, n)
    B = 2048
    pq = F.scenario_loads(f, np.arange(B))
    L = _lib.load()
    L.fpf_wave_rtc_builds.restype = C.c_int
    n0 = L.fpf_wave_rtc_builds()
    dev = torch.device("cuda:0")
    res = []
    for spec in (True, False):
        pf = PowerFlow(f, specialize=spec)
        assert pf.kernel == "wave" and pf.info["tile"] == 1
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
    assert L.fpf_wave_rtc_builds() >= max(n0, 1)   # (here or by an earlier test of the same plan)
    for k in res[0]:
        np.testing.assert_array_equal(res[0][k], res[1][k], err_msg=k)
    c = O.dpf_batch(f.Dl, f.Z, pq[:, :, :24], nthreads=8)
    conv = c["status"] == 0
    assert (res[0]["iters"][:24] == c["iters"]).all()
    assert _vrel(res[0]["v_re"][..., :24][..., conv], res[0]["v_im"][..., :24][..., conv], c["V_re"][..., conv],
                 c["V_im"][..., conv]) <= 1e-10
