"""GPU parity tests: libfreedm_pf (gfx950 kernels, through the C ABI) against the
oracle on the same inputs.

Bar (north_star): bus voltages within 1e-10 relative of the reference path and
identical iteration counts -- asserted for every kernel and mode.

Exact mode (fpf_opts.exact = 1; the generic and interpreted kernels always):
the kernels perform the reference's operations in the reference's order with
FMA contraction off, so the stronger checks also hold: complex V, PQb, PQL and
loss are bit-identical to the oracle; only results that pass through
hypot/atan (Vpolar, Vmin/Vmax) may differ by a few ulp (ocml vs glibc) --
tolerance 1e-14 relative (angles 1e-12 degrees).

Fast mode (the default of the specialised kernel): load currents as
conj(S)V/|V|^2 and FMA branch products, a few ulp per operation; checked at
the north-star bar plus PQb/PQL/Vpolar at 1e-9 and the loss at 1e-8 relative
(the loss is P_sub - sum P_load: cancellation amplifies rounding ~10-40x).
"""
import numpy as np
import pytest

from conftest import GOLDEN_NAMES, load_golden
from freedm_amd import feeder as F

pytestmark = pytest.mark.gpu

WF = {"g1_demo", "g1_demo_batch", "g2_dlnew", "g3_123bus", "g4_2048bus", "g5_nonconv", "g6_missing_phase"}


def _pf(Dl, Z, **kw):
    from freedm_amd import PowerFlow
    return PowerFlow(F.Feeder(Dl, Z), **kw)


def _vrel(a_re, a_im, b_re, b_im):
    a = a_re + 1j * a_im
    b = b_re + 1j * b_im
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300)))


KERNELS = [("generic", False, 1), ("tiled", False, 1), ("tiled", True, 1), ("tiled", True, 0), ("wave", False, 0)]


def _close(a, b, rtol):
    """|a - b| <= rtol * max|b| (per array: relative to the field's scale)."""
    scale = max(float(np.max(np.abs(b))), 1e-300)
    assert float(np.max(np.abs(a - b))) <= rtol * scale, (float(np.max(np.abs(a - b))), scale)


@pytest.mark.parametrize("kernel,spec,exact", KERNELS, ids=["generic", "tiled", "tiled-rtc", "tiled-rtc-fast", "wave"])
@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_matches_golden(name, kernel, spec, exact):
    g = load_golden(name)
    # the 2048-bus feeder is above the tiled hipRTC build's size limit: the build
    # is declined and the interpreted tiled kernel runs (same results)
    declined = kernel == "tiled" and name == "g4_2048bus" and spec
    pf = _pf(g["Dl"], g["Z"], kernel=kernel, specialize=spec, exact=exact)
    assert pf.kernel == kernel
    if kernel == "tiled":
        assert pf.info["specialized"] == (0 if declined else int(spec)), pf.rtc_error
    r = pf.solve(g["pq"])
    # the north-star bar
    assert (r["iters"] == g["iters"]).all()
    assert (r["status"] == g["status"]).all()
    conv = g["status"] == 0
    # on converged scenarios; a non-converged solve (G5: the reference throws) runs 20
    # sweeps of a diverging iteration, where fast-mode rounding grows
    assert _vrel(r["V_re"][..., conv], r["V_im"][..., conv], g["V_re"][..., conv], g["V_im"][..., conv]) <= 1e-10
    if exact:
        assert _vrel(r["V_re"], r["V_im"], g["V_re"], g["V_im"]) <= 1e-10
    else:
        _close(r["loss"][conv], g["loss"][conv], 1e-8)
        np.testing.assert_allclose(r["vmin"][conv], g["vmin"][conv], rtol=1e-10)
        np.testing.assert_allclose(r["vmax"][conv], g["vmax"][conv], rtol=1e-10)
        # whole batches (the fixtures keep 4 scenarios of the matrix outputs): the
        # oracle recomputes Vpolar / PQb / PQL for every converged scenario
        from oracle import oracle as O
        c = O.dpf_batch(g["Dl"], g["Z"], g["pq"], nthreads=8)
        _fast_mode_outputs_match(r, c, conv)
        return
    # the stronger claim: same operations, same order -> same bits
    np.testing.assert_array_equal(r["V_re"], g["V_re"])
    np.testing.assert_array_equal(r["V_im"], g["V_im"])
    np.testing.assert_array_equal(r["PQb"][:, :, :4], g["PQb"])
    np.testing.assert_array_equal(r["PQL"][:, :, :4], g["PQL"])
    np.testing.assert_array_equal(r["loss"], g["loss"])
    # hypot / atan: ocml vs glibc, a few ulp
    np.testing.assert_allclose(r["Vpolar"][0::2, :, :4], g["Vpolar"][0::2], rtol=1e-14, atol=0)
    np.testing.assert_allclose(r["Vpolar"][1::2, :, :4], g["Vpolar"][1::2], rtol=0, atol=1e-12)
    np.testing.assert_allclose(r["vmin"], g["vmin"], rtol=1e-14)
    np.testing.assert_allclose(r["vmax"], g["vmax"], rtol=1e-14)


def _fast_mode_outputs_match(r, c, conv):
    """Fast-mode matrix outputs against the oracle on the converged scenarios:
    PQb / PQL within 1e-9 of each field's scale, |V| within 1e-10 relative, and
    the angles (DPF_return7.cpp:231-235, atan of imag/real in degrees) within
    1e-8 deg -- V is within 1e-10 relative, so an angle moves by at most ~6e-9
    deg; a zeroed phase must read exactly the reference's -180 / +180 pattern."""
    _close(r["PQb"][..., conv], c["PQb"][..., conv], 1e-9)
    _close(r["PQL"][..., conv], c["PQL"][..., conv], 1e-9)
    mag_r, mag_c = r["Vpolar"][0::2][..., conv], c["Vpolar"][0::2][..., conv]
    np.testing.assert_allclose(mag_r, mag_c, rtol=1e-10, atol=0)
    ang_r, ang_c = r["Vpolar"][1::2][..., conv], c["Vpolar"][1::2][..., conv]
    np.testing.assert_allclose(ang_r, ang_c, rtol=0, atol=1e-8)
    zero = mag_c == 0
    np.testing.assert_array_equal(mag_r[zero], 0.0)
    np.testing.assert_array_equal(ang_r[zero], ang_c[zero])


def test_wave_divergent_convergence_in_one_wavefront():
    """Scenarios sharing a wavefront converge at different sweeps (loads scaled
    0.05x .. 3x, interleaved): each keeps the state of its own last sweep while
    the wave sweeps on (DPF_return7.cpp:199-217 break), so iteration counts,
    V and the matrix outputs match the oracle scenario by scenario."""
    from oracle import oracle as O
    f = F.synthetic_feeder(123, 123)
    pq = F.scenario_loads(f, np.arange(256))
    scale = np.tile(np.array([0.05, 3.0, 0.4, 2.2, 1.0, 0.15, 2.8, 0.7]), 32)
    pq = np.ascontiguousarray(pq * scale[None, None, :])
    pf = _pf(f.Dl, f.Z, kernel="wave")
    r = pf.solve(pq)
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    assert len(np.unique(c["iters"])) >= 3, np.unique(c["iters"])
    assert (r["iters"] == c["iters"]).all() and (r["status"] == c["status"]).all()
    conv = c["status"] == 0
    assert _vrel(r["V_re"][..., conv], r["V_im"][..., conv], c["V_re"][..., conv], c["V_im"][..., conv]) <= 1e-10
    _fast_mode_outputs_match(r, c, conv)
    _close(r["loss"][conv], c["loss"][conv], 1e-8)


def test_aggregates_on_two_streams():
    """Two aggregating solves of one feeder in flight on two streams (they share
    the feeder's partials / ticket scratch, which the library orders): both
    aggregates are right."""
    import torch
    f = F.synthetic_feeder(123, 123)
    pf = _pf(f.Dl, f.Z)
    dev = torch.device("cuda:0")
    B = 8192
    pqs = [F.scenario_loads(f, np.arange(i * B, (i + 1) * B)) for i in range(2)]
    host = [pf.solve(p)["aggregate"] for p in pqs]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    d_pq = [torch.from_numpy(p).to(dev) for p in pqs]
    aggs = [torch.zeros(8, dtype=torch.float64, device=dev) for _ in range(2)]
    outs = [{"loss": torch.zeros(B, dtype=torch.float64, device=dev)} for _ in range(2)]
    torch.cuda.synchronize()
    for rep in range(20):
        for i in (0, 1):
            pf.solve_device(d_pq[i], outs[i], agg=aggs[i], stream=streams[i])
        torch.cuda.synchronize()
        for i in (0, 1):
            a = aggs[i].cpu().numpy()
            h = host[i]
            assert a[3] == h["n_conv"] and a[7] == h["n_scen"] and a[1] == h["vmin"] and a[2] == h["vmax"], (rep, i)
            assert a[0] == pytest.approx(h["loss_sum"], rel=1e-12)


def test_auto_kernel_choice():
    g = load_golden("g3_123bus")
    assert _pf(g["Dl"], g["Z"]).kernel == "wave"            # fast mode (default)
    assert _pf(g["Dl"], g["Z"], exact=1).kernel == "tiled"  # the reference's roundings
    g4 = load_golden("g4_2048bus")
    pf4 = _pf(g4["Dl"], g4["Z"])                            # fast mode above 256 branches: the wave-block
    assert pf4.kernel == "wave" and pf4.info["tile"] == 1    # kernel, one scenario per workgroup
    assert _pf(g4["Dl"], g4["Z"], exact=1).kernel == "generic"   # exact: above the tiled kernel's size, tile 1
    f = F.demo_feeder()
    Dl = f.Dl[[0, 2, 1, 3, 4, 5, 6, 7, 8]].copy()     # 2->3 before 1->2: legal for the reference, not well formed
    pf = _pf(Dl, f.Z)                                   # fast mode: the wave kernel's sequential-order plan
    assert pf.kernel == "wave" and pf.info["well_formed"] == 0
    assert _pf(Dl, f.Z, exact=1).kernel == "generic"    # exact mode: the generic kernel
    from freedm_amd import DPFError
    with pytest.raises(DPFError):
        _pf(Dl, f.Z, kernel="tiled")
    with pytest.raises(DPFError):
        _pf(g["Dl"], g["Z"], kernel="wave", exact=1)


def test_malformed_order_matches_oracle():
    from oracle import oracle as O
    f = F.demo_feeder()
    Dl = f.Dl[[0, 2, 1, 3, 4, 5, 6, 7, 8]].copy()     # forward reads V(2) of the previous sweep
    pq = F.scenario_loads(F.Feeder(Dl, f.Z), np.arange(40))
    r = _pf(Dl, f.Z, exact=1).solve(pq)                # the generic kernel: the oracle's bits
    c = O.dpf_batch(Dl, f.Z, pq, nthreads=4)
    assert (r["iters"] == c["iters"]).all() and (r["status"] == c["status"]).all()
    np.testing.assert_array_equal(r["V_re"], c["V_re"])
    np.testing.assert_array_equal(r["V_im"], c["V_im"])
    r = _pf(Dl, f.Z).solve(pq)                          # fast mode: the wave kernel (tests/test_gpu_lag.py)
    assert (r["iters"] == c["iters"]).all() and (r["status"] == c["status"]).all()
    assert _vrel(r["V_re"], r["V_im"], c["V_re"], c["V_im"]) <= 1e-10


@pytest.mark.parametrize("spec", [False, True], ids=["interp", "rtc"])
@pytest.mark.parametrize("tile", [1, 3, 5, 8])
def test_tiles_and_ragged_batches(tile, spec):
    g = load_golden("g3_123bus")
    ref = _pf(g["Dl"], g["Z"], kernel="generic").solve(g["pq"][:, :, :13])
    r = _pf(g["Dl"], g["Z"], kernel="tiled", tile=tile, specialize=spec, exact=1).solve(g["pq"][:, :, :13])
    for k in ("V_re", "V_im", "PQb", "PQL", "Vpolar", "iters", "status", "loss", "vmin", "vmax"):
        np.testing.assert_array_equal(r[k], ref[k], err_msg=k)


def test_empty_and_single():
    g = load_golden("g1_demo")
    pf = _pf(g["Dl"], g["Z"])
    r0 = pf.solve(np.zeros((6, pf.nl, 0)))
    assert r0["iters"].size == 0 and r0["n_nonconv"] == 0
    r1 = pf.solve(g["pq"])   # default: the fast-mode wave kernel
    assert pf.kernel == "wave"
    assert _vrel(r1["V_re"], r1["V_im"], g["V_re"], g["V_im"]) <= 1e-10
    assert (r1["iters"] == g["iters"]).all()
    r2 = _pf(g["Dl"], g["Z"], exact=1).solve(g["pq"])   # the reference's roundings
    np.testing.assert_array_equal(r2["V_re"], g["V_re"])


def test_dpf_return7_dropin():
    from freedm_amd import DPF_return7, NonConvergedError
    from oracle import oracle as O
    f = F.demo_feeder()
    vpq = DPF_return7(f.Dl, f.Z)          # default: exact mode, the reference's roundings
    c = O.dpf_solve(f.Dl, f.Z)
    assert vpq.iters == c["iters"] == 5
    np.testing.assert_array_equal(vpq.PQb, c["PQb"])
    np.testing.assert_array_equal(vpq.PQL, c["PQL"])
    np.testing.assert_allclose(vpq.Vpolar, c["Vpolar"], rtol=1e-14, atol=1e-12)
    np.testing.assert_array_equal(vpq.Qset_b[:, 0], f.Dl[:, 9])
    fast = DPF_return7(f.Dl, f.Z, exact=False)
    assert fast.iters == 5
    _close(fast.PQb, c["PQb"], 1e-9)
    np.testing.assert_allclose(fast.Vpolar, c["Vpolar"], rtol=1e-10, atol=1e-8)
    g = load_golden("g5_nonconv")
    Dl = g["Dl"].copy()
    with pytest.raises(NonConvergedError):
        DPF_return7(Dl, g["Z"])


def test_bad_feeders_raise_topology_error():
    from freedm_amd import DPFError
    f = F.demo_feeder()
    for Dl in (np.vstack([f.Dl, np.zeros((1, 13))]), np.delete(f.Dl, 5, axis=0)):
        with pytest.raises(DPFError) as e:
            _pf(Dl, f.Z)
        assert e.value.code == -2


def test_full_config2_properties():
    """BASELINE config 2 at full size (123-bus, 4096 scenarios): size-independent
    properties -- the two kernels agree bit for bit, the fused loss equals the
    reference formula recomputed from PQb/PQL, the aggregate matches, and the
    solve is deterministic."""
    f = F.synthetic_feeder(123, 123)
    pq = F.scenario_loads(f, np.arange(4096))
    t = _pf(f.Dl, f.Z, kernel="tiled", exact=1)
    assert t.info["specialized"] == 1, t.rtc_error
    gen = _pf(f.Dl, f.Z, kernel="generic")
    interp = _pf(f.Dl, f.Z, kernel="tiled", specialize=False)
    a = t.solve(pq)
    b = gen.solve(pq)
    c3 = interp.solve(pq)
    a2 = t.solve(pq)
    for k in ("V_re", "V_im", "PQb", "PQL", "iters", "status", "loss", "vmin", "vmax"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
        np.testing.assert_array_equal(a[k], c3[k], err_msg=k)
        np.testing.assert_array_equal(a[k], a2[k], err_msg=k)
    assert (a["status"] == 0).all()
    # loss = accu([PQb(0,2p) - sum(PQL.col(2p))]) in Armadillo's order
    nn = t.nn
    x = []
    for p in range(3):
        col = a["PQL"][2 * p]
        acc1 = np.zeros(4096)
        acc2 = np.zeros(4096)
        for k in range(nn):
            if k & 1:
                acc2 = acc2 + col[k]
            else:
                acc1 = acc1 + col[k]
        x.append(a["PQb"][2 * p, 0] - (acc1 + acc2))
    np.testing.assert_array_equal(a["loss"], ((0.0 + x[0]) + x[2]) + (0.0 + x[1]))
    ag = a["aggregate"]
    conv = a["status"] == 0
    assert ag["n_conv"] == conv.sum() and ag["n_scen"] == 4096
    assert ag["vmin"] == a["vmin"][conv].min() and ag["vmax"] == a["vmax"][conv].max()
    assert ag["loss_sum"] == pytest.approx(a["loss"][conv].sum(), rel=1e-12)
    assert ag["n_under"] == (a["vmin"][conv] < 0.96).sum() and ag["n_over"] == (a["vmax"][conv] > 1.05).sum()
    # a sample against the oracle
    from oracle import oracle as O
    idx = np.arange(0, 4096, 97)
    c = O.dpf_batch(f.Dl, f.Z, pq[:, :, idx], nthreads=8)
    np.testing.assert_array_equal(a["V_re"][:, :, idx], c["V_re"])
    np.testing.assert_array_equal(a["iters"][idx], c["iters"])


@pytest.mark.parametrize("kernel", ["wave", "tiled"])
def test_fast_mode_full_batches_against_oracle(kernel):
    """The fast-mode kernels (the wave kernel is the default) against the oracle
    on whole batches: config 2 (4096 scenarios) and a 32768-scenario slice of the
    config-4 hosting study -- identical iteration counts and status everywhere,
    V within 1e-10."""
    from oracle import oracle as O
    f = F.synthetic_feeder(123, 123)
    pf = _pf(f.Dl, f.Z, kernel=kernel)
    assert pf.kernel == kernel
    if kernel == "tiled":
        assert pf.info["specialized"] == 1, pf.rtc_error
    for pq in (F.scenario_loads(f, np.arange(4096)), F.hosting_loads(f, np.arange(32768))):
        r = pf.solve(pq)
        c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=16)
        assert (r["iters"] == c["iters"]).all() and (r["status"] == c["status"]).all()
        assert _vrel(r["V_re"], r["V_im"], c["V_re"], c["V_im"]) <= 1e-10
        _close(r["loss"], c["loss"], 1e-8)
        np.testing.assert_allclose(r["vmin"], c["vmin"], rtol=1e-10)


def test_config4_wave_full_size():
    """BASELINE config 4 at the size the bench runs it: one GPU's 131 072-scenario
    shard of the hosting study (seed 2^20), scenario major, in one launch of the
    wave kernel with light outputs (V + scalars) and the fused aggregate; every
    scenario against the exact generic kernel on the same device inputs
    (iteration counts and status identical, V 1e-10, loss 1e-8, Vmin/Vmax 1e-10,
    the aggregate's counts equal) and a strided sample against the oracle
    (DPF_return7.cpp:199-217: the sweep count is the reference's)."""
    import torch
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    f = F.synthetic_feeder(123, 123)
    B = 131072
    dev = torch.device("cuda:0")
    d_pq = torch.empty((B, 6, f.nl), dtype=torch.float64, device=dev)
    for a in range(0, B, 16384):
        d_pq[a:a + 16384] = torch.from_numpy(
            F.hosting_loads(f, np.arange(a, a + 16384), seed=1 << 20).transpose(2, 0, 1).copy()).to(dev)

    def run(pf):
        nn = pf.nn
        out = {"v_re": torch.empty((B, 3, nn), dtype=torch.float64, device=dev),
               "v_im": torch.empty((B, 3, nn), dtype=torch.float64, device=dev),
               "iters": torch.empty(B, dtype=torch.int32, device=dev),
               "status": torch.empty(B, dtype=torch.int8, device=dev),
               "loss": torch.empty(B, dtype=torch.float64, device=dev),
               "vmin": torch.empty(B, dtype=torch.float64, device=dev),
               "vmax": torch.empty(B, dtype=torch.float64, device=dev)}
        agg = torch.zeros(8, dtype=torch.float64, device=dev)
        pf.solve_device(d_pq, out, agg=agg)
        torch.cuda.synchronize()
        return out, agg.cpu().numpy()

    fast = PowerFlow(f, device=0, layout=1)
    assert fast.kernel == "wave"
    w, wa = run(fast)
    assert wa[7] == B and wa[3] + wa[4] == B
    it = w["iters"].cpu().numpy()
    assert len(set(it.tolist())) >= 2   # mixed sweep counts within wavefronts
    idx = np.arange(0, B, 1021)
    ti = torch.from_numpy(idx).to(dev)
    pq_s = np.ascontiguousarray(d_pq[ti].cpu().numpy().transpose(1, 2, 0))
    c = O.dpf_batch(f.Dl, f.Z, pq_s, nthreads=8)
    assert (it[idx] == c["iters"]).all() and (w["status"][ti].cpu().numpy() == c["status"]).all()
    vr = np.moveaxis(w["v_re"][ti].cpu().numpy(), 0, -1)
    vi = np.moveaxis(w["v_im"][ti].cpu().numpy(), 0, -1)
    assert _vrel(vr, vi, c["V_re"], c["V_im"]) <= 1e-10
    _close(w["loss"][ti].cpu().numpy(), c["loss"], 1e-8)
    np.testing.assert_allclose(w["vmin"][ti].cpu().numpy(), c["vmin"], rtol=1e-10)
    np.testing.assert_allclose(w["vmax"][ti].cpu().numpy(), c["vmax"], rtol=1e-10)
    exact = PowerFlow(f, device=0, exact=1, layout=1)   # (a batch this size runs the generic kernel)
    g, ga = run(exact)
    assert torch.equal(w["iters"], g["iters"]) and torch.equal(w["status"], g["status"])
    for c0 in range(0, B, 32768):   # (in chunks: complex V of the whole shard is 0.8 GB per kernel)
        a = torch.complex(w["v_re"][c0:c0 + 32768], w["v_im"][c0:c0 + 32768])
        b = torch.complex(g["v_re"][c0:c0 + 32768], g["v_im"][c0:c0 + 32768])
        assert float(((a - b).abs() / b.abs()).max()) <= 1e-10
        del a, b
    assert float(((w["loss"] - g["loss"]).abs() / g["loss"].abs().max()).max()) <= 1e-8
    assert float(((w["vmin"] - g["vmin"]).abs() / g["vmin"]).max()) <= 1e-10
    assert float(((w["vmax"] - g["vmax"]).abs() / g["vmax"]).max()) <= 1e-10
    np.testing.assert_array_equal(wa[3:], ga[3:])
    np.testing.assert_allclose(wa[:3], ga[:3], rtol=1e-8)


def test_device_api_on_torch_stream():
    import torch
    f = F.synthetic_feeder(123, 123)
    pq = F.scenario_loads(f, np.arange(1000))
    pf = _pf(f.Dl, f.Z)
    host = pf.solve(pq)
    dev = torch.device("cuda:0")
    d_pq = torch.from_numpy(pq).to(dev)
    B = pq.shape[2]
    out = {"iters": torch.zeros(B, dtype=torch.int32, device=dev), "status": torch.zeros(B, dtype=torch.int8, device=dev),
           "loss": torch.zeros(B, dtype=torch.float64, device=dev), "vmin": torch.zeros(B, dtype=torch.float64, device=dev),
           "vmax": torch.zeros(B, dtype=torch.float64, device=dev),
           "v_re": torch.zeros((3, pf.nn, B), dtype=torch.float64, device=dev),
           "v_im": torch.zeros((3, pf.nn, B), dtype=torch.float64, device=dev)}
    agg = torch.zeros(8, dtype=torch.float64, device=dev)
    pf.solve_device(d_pq, out, agg=agg, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["v_re"].cpu().numpy(), host["V_re"])
    np.testing.assert_array_equal(out["loss"].cpu().numpy(), host["loss"])
    np.testing.assert_array_equal(out["iters"].cpu().numpy(), host["iters"])
    assert agg.cpu().numpy()[3] == host["aggregate"]["n_conv"]


def test_hosting_shards_are_invariant():
    """Config 4 partitioning: a scenario's result does not depend on which shard
    (GPU) solved it (seeds derive from the global scenario index)."""
    f = F.synthetic_feeder(123, 123)
    pf = _pf(f.Dl, f.Z)
    full = pf.solve(F.hosting_loads(f, np.arange(512)))
    lo = pf.solve(F.hosting_loads(f, np.arange(0, 256)))
    hi = pf.solve(F.hosting_loads(f, np.arange(256, 512)))
    np.testing.assert_array_equal(np.concatenate([lo["V_re"], hi["V_re"]], axis=2), full["V_re"])
    np.testing.assert_array_equal(np.concatenate([lo["loss"], hi["loss"]]), full["loss"])


def test_shared_reciprocal_division_is_bit_exact():
    """The tiled kernel's dv_div / cdiv_rr (fpf_math.hpp) against the compiler's
    a / b and libgcc's __divdc3, bit for bit, on 2^26 seeded operand sets over
    the guarded exponent range, zeros and signs included."""
    from freedm_amd import _lib
    assert _lib.load().fpf_selftest_division(0, 1 << 26, 20261016) == 0


@pytest.mark.parametrize("tracks", [1, 2, 3, 4])
def test_track_counts_are_bit_identical(tracks, monkeypatch):
    """Every multi-track schedule of the specialised kernel (fpf_api.cpp:
    schedule_tracks) gives the reference's bits: V, PQb, PQL, loss, iterations."""
    monkeypatch.setenv("FPF_RTC_TRACKS", str(tracks))
    for name in ("g1_demo_batch", "g2_dlnew", "g3_123bus", "g5_nonconv", "g6_missing_phase"):
        g = load_golden(name)
        pf = _pf(g["Dl"], g["Z"], kernel="tiled", specialize=True, exact=1)
        assert pf.info["specialized"] == 1, pf.rtc_error
        r = pf.solve(g["pq"])
        assert (r["iters"] == g["iters"]).all() and (r["status"] == g["status"]).all(), name
        np.testing.assert_array_equal(r["V_re"], g["V_re"], err_msg=name)
        np.testing.assert_array_equal(r["V_im"], g["V_im"], err_msg=name)
        np.testing.assert_array_equal(r["PQb"][:, :, :4], g["PQb"], err_msg=name)
        np.testing.assert_array_equal(r["PQL"][:, :, :4], g["PQL"], err_msg=name)
        np.testing.assert_array_equal(r["loss"], g["loss"], err_msg=name)


def test_config3_full_size_against_oracle():
    """BASELINE config 3 at its stated size in exact mode: the 2048-bus feeder,
    65 536 scenarios in one batch (exact mode at this batch size = the generic
    kernel; fast mode, the wave-block kernel, in tests/test_gpu_wblk.py).  The batch is built on the GPU from 1 024 seeded base scenarios
    (config-3 generator, seed 65536) times a per-scenario multiplier, so all
    65 536 differ; a strided sample of 65 scenarios is recomputed by the oracle
    with the same inputs: identical iteration counts and status, V bit-identical
    (the generic kernel is exact mode) and within the 1e-10 bar."""
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
    pf = PowerFlow(f, device=0, exact=1)
    assert pf.kernel == "generic"
    nn = pf.nn
    out = {"v_re": torch.empty((3, nn, B), dtype=torch.float64, device=dev),
           "v_im": torch.empty((3, nn, B), dtype=torch.float64, device=dev),
           "iters": torch.empty(B, dtype=torch.int32, device=dev), "status": torch.empty(B, dtype=torch.int8, device=dev),
           "loss": torch.empty(B, dtype=torch.float64, device=dev), "vmin": torch.empty(B, dtype=torch.float64, device=dev),
           "vmax": torch.empty(B, dtype=torch.float64, device=dev)}
    agg = torch.zeros(8, dtype=torch.float64, device=dev)
    pf.solve_device(d_pq, out, agg=agg)
    torch.cuda.synchronize()
    a = agg.cpu().numpy()
    assert a[7] == B and a[3] + a[4] == B
    idx = np.arange(0, B, 1021)
    ti = torch.from_numpy(idx).to(dev)
    pq_s = np.ascontiguousarray(base[:, :, idx % NB] * mult[idx])
    c = O.dpf_batch(f.Dl, f.Z, pq_s, nthreads=8)
    it = out["iters"][ti].cpu().numpy()
    st = out["status"][ti].cpu().numpy()
    assert (it == c["iters"]).all() and (st == c["status"]).all()
    v_re = out["v_re"][:, :, ti].cpu().numpy()
    v_im = out["v_im"][:, :, ti].cpu().numpy()
    assert _vrel(v_re, v_im, c["V_re"], c["V_im"]) <= 1e-10
    np.testing.assert_array_equal(v_re, c["V_re"])
    np.testing.assert_array_equal(v_im, c["V_im"])
    np.testing.assert_array_equal(out["loss"][ti].cpu().numpy(), c["loss"])


def test_overlapping_outputs_refused():
    """fpf_outputs arrays must not overlap (include/freedm_pf.h: the fast kernels
    stash a scenario's IL / Ib in its own pql / pqb entries): overlapping ranges
    are refused with FPF_ERR_ARG before anything is enqueued, and a call with
    disjoint views of one allocation still solves."""
    import torch
    from freedm_amd import DPFError, PowerFlow
    f = F.synthetic_feeder(123, 123)
    B = 64
    pq = torch.from_numpy(F.scenario_loads(f, np.arange(B), seed=7)).to("cuda:0")
    pf = PowerFlow(f, device=0)
    nn = pf.nn
    big = torch.empty((2, 6, nn, B), dtype=torch.float64, device="cuda:0")
    with pytest.raises(DPFError):
        pf.solve_device(pq, {"pqb": big[0], "pql": big[0]})
    with pytest.raises(DPFError):   # a partial overlap: pql starts inside pqb
        flat = big.reshape(-1)
        pf.solve_device(pq, {"pqb": flat[: 6 * nn * B].view(6, nn, B),
                             "pql": flat[nn * B: nn * B + 6 * nn * B].view(6, nn, B)})
    out = {"pqb": big[0], "pql": big[1], "iters": torch.empty(B, dtype=torch.int32, device="cuda:0")}
    pf.solve_device(pq, out)
    torch.cuda.synchronize()
    assert int(out["iters"].min()) >= 1
