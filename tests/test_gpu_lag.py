"""The wave kernel's sequential-order plan on the GPU (fpf_api.cpp:
analyse_wave_lag, fpf_wave_body.h under f.has_lag): Dl tables whose rows do not
follow the feeder tree -- laterals listed before their taps' rows, rows inside a
block that do not chain, branches fed from a node whose row comes later -- which
the reference solves with its sequential semantics (DPF_return7.cpp:134-195).
They used to run only on the exact generic kernel (~10x slower); fast mode now
runs them on the wave kernel, checked against the oracle at the north-star bar:
identical iteration counts and status, V within 1e-10 relative, PQb / PQL /
Vpolar as tests/test_gpu_parity.py's fast-mode bar, loss 1e-8, Vmin/Vmax 1e-10;
zeroed phases in such tables too (lag_tables.zeroed_cases)."""
import numpy as np
import pytest

from freedm_amd import feeder as F
from lag_tables import cases, restart_cases, wblk_cases, zeroed_cases
from test_gpu_parity import _close, _fast_mode_outputs_match, _vrel

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(cases()))
def test_sequential_order_tables_on_the_wave_kernel(name):
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    f = cases()[name]
    B = 192
    pq = F.scenario_loads(f, np.arange(B))
    pf = PowerFlow(f)
    assert pf.kernel == "wave", pf.info
    r = pf.solve(pq)
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    np.testing.assert_array_equal(r["iters"], c["iters"])
    np.testing.assert_array_equal(r["status"], c["status"])
    conv = c["status"] == 0
    assert conv.all()
    assert _vrel(r["V_re"], r["V_im"], c["V_re"], c["V_im"]) <= 1e-10
    _fast_mode_outputs_match(r, c, conv)
    _close(r["loss"], c["loss"], 1e-8)
    np.testing.assert_allclose(r["vmin"], c["vmin"], rtol=1e-10)
    np.testing.assert_allclose(r["vmax"], c["vmax"], rtol=1e-10)
    # exact mode: the generic kernel (the tiled one where the table is well formed), the oracle's bits
    e = PowerFlow(f, exact=1)
    assert e.kernel in ("generic", "tiled")
    re_ = e.solve(pq[:, :, :16])
    np.testing.assert_array_equal(re_["V_re"], c["V_re"][..., :16])


@pytest.mark.parametrize("name", sorted(zeroed_cases()))
def test_sequential_order_zeroed_phases_on_the_wave_kernel(name):
    """Sequential-order tables with zeroed phases (V = 0 on them, IL = 0 there,
    DPF_return7.cpp:180-192; one whose rows below a zeroed node read its
    previous-sweep V) on the wave kernel's FULL variant with both general paths:
    the same bar."""
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    f = zeroed_cases()[name]
    B = 192
    pq = F.scenario_loads(f, np.arange(B), pv_frac=0.0)
    pf = PowerFlow(f)
    assert pf.kernel == "wave", pf.info
    r = pf.solve(pq)
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    np.testing.assert_array_equal(r["iters"], c["iters"])
    np.testing.assert_array_equal(r["status"], c["status"])
    conv = c["status"] == 0
    assert conv.all()
    assert (c["V_re"] == 0).any()   # some (node, phase) zeroed
    assert _vrel(r["V_re"], r["V_im"], c["V_re"], c["V_im"]) <= 1e-10   # zeroed entries: exactly 0 in both
    _fast_mode_outputs_match(r, c, conv)
    _close(r["loss"], c["loss"], 1e-8)
    np.testing.assert_allclose(r["vmin"], c["vmin"], rtol=1e-10)
    np.testing.assert_allclose(r["vmax"], c["vmax"], rtol=1e-10)
    e = PowerFlow(f, exact=1)
    re_ = e.solve(pq[:, :, :16])
    np.testing.assert_array_equal(re_["V_re"], c["V_re"][..., :16])


@pytest.mark.parametrize("name", sorted(restart_cases()))
def test_restart_below_zeroed_runs_generic(name):
    """A live phase restarting below a zeroed node in sequential order: the plan
    declines it and fast mode runs the generic kernel -- the oracle's V, iteration
    counts and status."""
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    f = restart_cases()[name]
    pq = F.scenario_loads(f, np.arange(48), pv_frac=0.0)
    pf = PowerFlow(f)
    assert pf.kernel == "generic", pf.info
    r = pf.solve(pq)
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    np.testing.assert_array_equal(r["iters"], c["iters"])
    np.testing.assert_array_equal(r["status"], c["status"])
    assert _vrel(r["V_re"], r["V_im"], c["V_re"], c["V_im"]) <= 1e-10


@pytest.mark.parametrize("name", sorted(wblk_cases()))
def test_sequential_order_tables_on_the_wave_block_kernel(name):
    """Past 256 branches (fpf_wblk_body.h under f.has_lag): the same bar."""
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    f = wblk_cases()[name]
    B = 96
    pq = F.scenario_loads(f, np.arange(B))
    pf = PowerFlow(f)
    assert pf.kernel == "wave" and pf.info["tile"] == 1, pf.info
    r = pf.solve(pq)
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    np.testing.assert_array_equal(r["iters"], c["iters"])
    np.testing.assert_array_equal(r["status"], c["status"])
    assert (c["status"] == 0).all()
    assert _vrel(r["V_re"], r["V_im"], c["V_re"], c["V_im"]) <= 1e-10
    _fast_mode_outputs_match(r, c, c["status"] == 0)
    _close(r["loss"], c["loss"], 1e-8)
    np.testing.assert_allclose(r["vmin"], c["vmin"], rtol=1e-10)
    np.testing.assert_allclose(r["vmax"], c["vmax"], rtol=1e-10)


@pytest.mark.parametrize("name", ["123-shuffled1", "123-swapped", "700-shuffled-swapped", "123-shuffled-zeroed"])
def test_sequential_order_device_batches(name):
    """Device buffers, both layouts, a batch past the per-plan build's threshold
    (4096) and a ragged one: V and the scalars against the host-buffer solve's."""
    import torch
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    f = {**cases(), **wblk_cases(), **zeroed_cases()}[name]
    dev = torch.device("cuda:0")
    for B in (4103, 77):
        pq = F.scenario_loads(f, np.arange(B), pv_frac=0.0 if "zeroed" in name else 0.2)
        for layout in (0, 1):
            pf = PowerFlow(f, layout=layout)
            x = pq if layout == 0 else np.ascontiguousarray(pq.transpose(2, 0, 1))
            sh = (3, pf.nn, B) if layout == 0 else (B, 3, pf.nn)
            out = {"v_re": torch.zeros(sh, dtype=torch.float64, device=dev),
                   "v_im": torch.zeros(sh, dtype=torch.float64, device=dev),
                   "iters": torch.zeros(B, dtype=torch.int32, device=dev),
                   "status": torch.zeros(B, dtype=torch.int8, device=dev),
                   "loss": torch.zeros(B, dtype=torch.float64, device=dev),
                   "vmin": torch.zeros(B, dtype=torch.float64, device=dev)}
            pf.solve_device(torch.from_numpy(x).to(dev), out)
            torch.cuda.synchronize()
            r = {k: v.cpu().numpy() for k, v in out.items()}
            if layout == 1:
                r["v_re"], r["v_im"] = r["v_re"].transpose(1, 2, 0), r["v_im"].transpose(1, 2, 0)
            idx = np.arange(0, B, 37)
            c = O.dpf_batch(f.Dl, f.Z, pq[:, :, idx], nthreads=8)
            np.testing.assert_array_equal(r["iters"][idx], c["iters"])
            assert _vrel(r["v_re"][..., idx], r["v_im"][..., idx], c["V_re"], c["V_im"]) <= 1e-10
            _close(r["loss"][idx], c["loss"], 1e-8)
            np.testing.assert_allclose(r["vmin"][idx], c["vmin"], rtol=1e-10)
