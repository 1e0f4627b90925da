"""The paired wave-block kernel (fpf_wcoop.hip; fast mode on feeders of
2049..4096 branches, one scenario on two workgroups that exchange their scan
values every sweep) against the oracle and the exact generic kernel.

Bar (north_star, as for the other fast kernels): V within 1e-10 relative and
identical iteration counts and status on every scenario; PQb / PQL / Vpolar at
1e-9 (angles 1e-8 deg), loss 1e-8, Vmin/Vmax 1e-10.  The reference:
DPF_return7.cpp:8-263 (any Nl) and the VVC reductions (VoltVarCtrl.cpp:1152-1161,
1201-1207), restated by oracle/ref_dpf.c.
"""
import numpy as np
import pytest

from freedm_amd import feeder as F
from test_gpu_wblk import _check_full, _vrel

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [2100, 3000, 4096])
def test_wcoop_matches_oracle(n):
    """Full outputs (the FULL variant) against the oracle, scenario by scenario;
    the kernel is the paired one (the plan's 2 x 8 wavefronts)."""
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    f = F.synthetic_feeder(n, n)
    pq = F.scenario_loads(f, np.arange(24))
    pf = PowerFlow(f)
    assert pf.kernel == "wave" and pf.info["tile"] == 1
    r = pf.solve(pq)
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    assert (c["status"] == 0).all()
    _check_full(r, c)


def test_wcoop_mixed_sweeps_both_layouts():
    """Loads scaled 0.05x .. 40x on the 4096-bus feeder: different sweep counts
    and non-convergent scenarios (status 1 after 20 sweeps) in one batch, the
    light outputs (V + scalars, device buffers) in both batch layouts, against
    the oracle."""
    import torch
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    f = F.synthetic_feeder(4096, 4096)
    B = 40
    pq = np.ascontiguousarray(F.scenario_loads(f, np.arange(B)) * np.geomspace(0.05, 40.0, B)[None, None, :])
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    assert (c["status"] == 1).any() and len(set(c["iters"][c["status"] == 0])) >= 3
    conv = c["status"] == 0
    dev = torch.device("cuda:0")
    for layout in (0, 1):
        pf = PowerFlow(f, layout=layout)
        x = pq if layout == 0 else np.ascontiguousarray(pq.transpose(2, 0, 1))
        sh = (3, pf.nn, B) if layout == 0 else (B, 3, pf.nn)
        o = {"v_re": torch.empty(sh, dtype=torch.float64, device=dev),
             "v_im": torch.empty(sh, dtype=torch.float64, device=dev),
             "iters": torch.empty(B, dtype=torch.int32, device=dev),
             "status": torch.empty(B, dtype=torch.int8, device=dev),
             "loss": torch.empty(B, dtype=torch.float64, device=dev),
             "vmin": torch.empty(B, dtype=torch.float64, device=dev),
             "vmax": torch.empty(B, dtype=torch.float64, device=dev)}
        pf.solve_device(torch.from_numpy(x).to(dev), o)
        torch.cuda.synchronize()
        r = {k: v.cpu().numpy() for k, v in o.items()}
        vr, vi = (r["v_re"], r["v_im"]) if layout == 0 else (np.moveaxis(r["v_re"], 0, -1), np.moveaxis(r["v_im"], 0, -1))
        assert (r["iters"] == c["iters"]).all() and (r["status"] == c["status"]).all()
        e = _vrel(vr[..., conv], vi[..., conv], c["V_re"][..., conv], c["V_im"][..., conv])
        print(f"layout {layout}: max V rel err {e:.3e}, sweeps {c['iters'][conv].min()}..{c['iters'][conv].max()}")
        assert e <= 1e-10
        np.testing.assert_allclose(r["vmin"][conv], c["vmin"][conv], rtol=1e-10)
        np.testing.assert_allclose(r["vmax"][conv], c["vmax"][conv], rtol=1e-10)
        np.testing.assert_allclose(r["loss"][conv], c["loss"][conv], rtol=1e-8)
        pf.close()


def test_wcoop_16384_scenarios():
    """16 384 scenarios of the 4096-bus feeder in one launch (light outputs and
    the fused aggregate; every exchange area reused 16 times): every scenario
    against the exact generic kernel on the same device inputs (iteration counts
    and status identical, V 1e-10, loss 1e-8, Vmin/Vmax 1e-10, the aggregate's
    counts equal) and a strided sample against the oracle."""
    import torch
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    f = F.synthetic_feeder(4096, 4096)
    B, NB = 16384, 512
    base = F.scenario_loads(f, np.arange(NB), seed=16384)
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
    assert fast.kernel == "wave"
    w, wa = run(fast)
    assert wa[7] == B and wa[3] == B
    idx = np.arange(0, B, 509)
    ti = torch.from_numpy(idx).to(dev)
    pq_s = np.ascontiguousarray(base[:, :, idx % NB] * mult[idx])
    c = O.dpf_batch(f.Dl, f.Z, pq_s, nthreads=8)
    assert (w["iters"][ti].cpu().numpy() == c["iters"]).all() and (w["status"][ti].cpu().numpy() == c["status"]).all()
    assert _vrel(w["v_re"][:, :, ti].cpu().numpy(), w["v_im"][:, :, ti].cpu().numpy(), c["V_re"], c["V_im"]) <= 1e-10
    np.testing.assert_allclose(w["loss"][ti].cpu().numpy(), c["loss"], rtol=1e-8)
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


def _single_phase_subtrees(n, seed):
    """Synthetic feeder whose laterals 3 and 7 are phase-B-only with everything
    below them (a phase-B-only line code on every row of the two subtrees, their
    phase-A and -C loads removed): zeroed phases without a live phase below a
    zeroed one -- the physical case (single-phase laterals)."""
    f = F.synthetic_feeder(n, seed)
    Dl = f.Dl.copy()
    Z = np.vstack([f.Z, np.diag([0, 0.3 + 0.8j, 0])])
    code = Z.shape[0] // 3
    seps = np.flatnonzero(Dl[:, 0] == 0)
    nn = int((Dl[:, 0] != 0).sum()) + 1
    kids = [[] for _ in range(nn)]
    row_of = {}
    for m in range(Dl.shape[0]):
        if Dl[m, 0] != 0:
            kids[0 if m == 0 else int(Dl[m, 1])].append(int(Dl[m, 2]))
            row_of[int(Dl[m, 2])] = m
    for i in (3, 7):
        st = [int(Dl[seps[i] + 1, 2])]
        while st:
            k = st.pop()
            Dl[row_of[k], 3] = code
            Dl[row_of[k], [6, 7, 10, 11]] = 0
            st.extend(kids[k])
    return F.Feeder(Dl, Z, name=f"synthetic-{n}bus-single-phase-laterals")


def _many_codes_feeder(n, seed, ncodes=70):
    """Synthetic feeder whose branches (row 0 aside) use `ncodes` distinct
    asymmetric line codes (code 1's 3x3 block with every entry perturbed by a
    seeded factor in [0.8, 1.2]): the paired kernel's per-code Zl table in its
    9-entry form, ncodes x 9 > 511 (the code field of its slot register holds the
    code index, not code x 9)."""
    f = F.synthetic_feeder(n, seed)
    rng = np.random.default_rng(seed + 1)
    z1 = f.Z[0:3]
    extra = [z1 * (0.8 + 0.4 * rng.random((3, 3))) for _ in range(ncodes)]
    Z = np.vstack([f.Z] + extra)
    Dl = f.Dl.copy()
    first = f.Z.shape[0] // 3 + 1
    br = np.flatnonzero(Dl[:, 0] != 0)[1:]
    Dl[br, 3] = first + (np.arange(br.size) % ncodes)
    return F.Feeder(Dl, Z, name=f"synthetic-{n}bus-{ncodes}codes")


def test_wcoop_many_asymmetric_codes():
    """70 asymmetric line codes on a 3000-bus feeder (Zl table 70 x 9 entries):
    the paired kernel against the oracle at the fast-mode bar."""
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    f = _many_codes_feeder(3000, 3000)
    pq = F.scenario_loads(f, np.arange(16))
    pf = PowerFlow(f)
    assert pf.kernel == "wave" and pf.info["tile"] == 1
    r = pf.solve(pq)
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    assert (c["status"] == 0).all()
    _check_full(r, c)


@pytest.mark.parametrize("n", [3000, 4096])
def test_wcoop_zeroed_phases(n):
    """Zeroed phases on the paired kernel (single-phase laterals: a phase-B-only
    line code on two laterals, DPF_return7.cpp:180-192): V = 0 on the zeroed
    phases and the -180/+180 angle pattern, the loss over PQL, the general
    V_abc_list extremes (Lnum_p + 1 < Nn: both workgroups' |V| ranked in node
    order), against the oracle at the fast-mode bar."""
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    from test_gpu_parity import _fast_mode_outputs_match
    from test_gpu_wblk import _close
    f = _single_phase_subtrees(n, n)
    pq = F.scenario_loads(f, np.arange(24), pv_frac=0.0)
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    assert (c["status"] == 0).all() and (c["Vpolar"][0::2] == 0).any()
    nn = int((f.Dl[:, 0] != 0).sum()) + 1
    assert min(O.lnum(f.Dl, f.Z)) + 1 < nn
    pf = PowerFlow(f)
    assert pf.kernel == "wave" and pf.info["tile"] == 1
    r = pf.solve(pq)
    assert (r["iters"] == c["iters"]).all() and (r["status"] == c["status"]).all()
    assert _vrel(r["V_re"], r["V_im"], c["V_re"], c["V_im"]) <= 1e-10
    _close(r["loss"], c["loss"], 1e-8)
    np.testing.assert_allclose(r["vmin"], c["vmin"], rtol=1e-10)
    np.testing.assert_allclose(r["vmax"], c["vmax"], rtol=1e-10)
    _fast_mode_outputs_match(r, c, c["status"] == 0)
    # the light outputs (V + scalars) on the device, scenario-major
    import torch
    dev = torch.device("cuda:0")
    pf1 = PowerFlow(f, layout=1)
    B = pq.shape[2]
    o = {"v_re": torch.empty((B, 3, pf1.nn), dtype=torch.float64, device=dev),
         "v_im": torch.empty((B, 3, pf1.nn), dtype=torch.float64, device=dev),
         "iters": torch.empty(B, dtype=torch.int32, device=dev),
         "loss": torch.empty(B, dtype=torch.float64, device=dev),
         "vmin": torch.empty(B, dtype=torch.float64, device=dev),
         "vmax": torch.empty(B, dtype=torch.float64, device=dev)}
    pf1.solve_device(torch.from_numpy(np.ascontiguousarray(pq.transpose(2, 0, 1))).to(dev), o)
    torch.cuda.synchronize()
    assert (o["iters"].cpu().numpy() == c["iters"]).all()
    vr, vi = np.moveaxis(o["v_re"].cpu().numpy(), 0, -1), np.moveaxis(o["v_im"].cpu().numpy(), 0, -1)
    assert _vrel(vr, vi, c["V_re"], c["V_im"]) <= 1e-10
    np.testing.assert_allclose(o["vmin"].cpu().numpy(), c["vmin"], rtol=1e-10)
    np.testing.assert_allclose(o["loss"].cpu().numpy(), c["loss"], rtol=1e-8)


def test_wcoop_declines_restart_and_larger_feeders():
    """A live phase below a zeroed one above 2048 branches and feeders above 4096
    branches stay on the generic kernel (bit-identical to the oracle in exact
    mode, its own tests)."""
    from freedm_amd import PowerFlow
    from test_gpu_wblk import _masked_feeder
    assert PowerFlow(_masked_feeder(3000, 3000, restart=True)).kernel == "generic"
    assert PowerFlow(F.synthetic_feeder(4300, 4300)).kernel == "generic"


def test_wcoop_areas_equal_monolithic():
    """The multi-area solve (fpf_areas_*: per-scenario source voltages, the
    children's source power, warm starts, the device-side stop) on a 3000-bus
    feeder whose root area needs the paired kernel: V equals the monolithic
    solve to 1e-10."""
    from freedm_amd import AreaPowerFlow
    from oracle import oracle as O
    f = F.synthetic_feeder(3000, 3000)
    Dl = f.Dl
    nn = int((Dl[:, 0] != 0).sum()) + 1
    kids = [[] for _ in range(nn)]
    for m in range(Dl.shape[0]):
        if Dl[m, 0] != 0:
            kids[0 if m == 0 else int(Dl[m, 1])].append(int(Dl[m, 2]))
    size = np.ones(nn, dtype=np.int64)
    for k in range(nn - 1, 0, -1):   # (children carry larger bus numbers on the synthetic feeder)
        for c in kids[k]:
            size[k] += size[c]
    # two disjoint subtrees of 80..300 buses as the child areas
    inside = np.zeros(nn, dtype=bool)
    tops = []
    for k in range(nn - 1, 0, -1):
        if len(tops) < 2 and 80 <= size[k] <= 300 and not inside[k]:
            st = [k]
            sub = []
            while st:
                x = st.pop()
                sub.append(x)
                st.extend(kids[x])
            if inside[sub].any():
                continue
            inside[sub] = True
            tops.append(k)
    assert len(tops) == 2
    node_area = F.subtree_node_areas(f, tops)
    assert (node_area == 0).sum() > 2049
    pq = F.scenario_loads(f, np.arange(16))
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


@pytest.mark.parametrize("B", [1, 9, 17])
def test_wcoop_small_and_ragged_batches(B):
    """Batches that leave padding pairs in the last group of 8 scenarios (the
    grid is 16 workgroups per 8 scenarios): every real scenario against the
    oracle, the padding members exit without touching an exchange area."""
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    f = F.synthetic_feeder(2100, 2100)
    pq = F.scenario_loads(f, np.arange(B))
    r = PowerFlow(f).solve(pq)
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=8)
    _check_full(r, c)


def test_wcoop_exchange_failure_reported(monkeypatch):
    """A paired-kernel hand-off that gives up (forced: FPF_TEST_COOP_SPIN = 0 polls,
    read at feeder creation) is its own outcome, never a non-convergence
    (DPF_return7.cpp:199-217 defines that): every scenario reports status
    FPF_EXCHANGE_FAILED (3), the aggregate counts none as converged or
    non-converged, the host entry returns FPF_ERR_EXCHANGE, and the device entry
    reports it through fpf_feeder_check and at the next call on the feeder."""
    import torch
    from freedm_amd import PowerFlow
    from freedm_amd.engine import ExchangeError, FPF_EXCHANGE_FAILED
    f = F.synthetic_feeder(2100, 2100)
    monkeypatch.setenv("FPF_TEST_COOP_SPIN", "0")
    pf = PowerFlow(f)
    monkeypatch.delenv("FPF_TEST_COOP_SPIN")
    assert pf.kernel == "wave"
    B = 9
    pq = F.scenario_loads(f, np.arange(B))
    with pytest.raises(ExchangeError) as ei:
        pf.solve(pq, full=False)
    r = ei.value.results
    assert ei.value.code == -6 and (r["status"] == FPF_EXCHANGE_FAILED).all()
    a = r["aggregate"]
    assert a["n_conv"] == 0 and a["n_nonconv"] == 0 and a["n_scen"] == B
    dev = torch.device("cuda:0")
    o = {"iters": torch.empty(B, dtype=torch.int32, device=dev), "status": torch.empty(B, dtype=torch.int8, device=dev),
         "loss": torch.empty(B, dtype=torch.float64, device=dev)}
    agg = torch.zeros(8, dtype=torch.float64, device=dev)
    d_pq = torch.from_numpy(pq).to(dev)
    pf.solve_device(d_pq, o, agg=agg)   # asynchronous: returns FPF_OK
    with pytest.raises(ExchangeError):
        pf.check()
    pf.check()                          # reported once
    assert (o["status"].cpu().numpy() == FPF_EXCHANGE_FAILED).all()
    ag = agg.cpu().numpy()
    assert ag[3] == 0 and ag[4] == 0 and ag[7] == B
    pf.solve_device(d_pq, o)
    torch.cuda.synchronize()
    with pytest.raises(ExchangeError):  # the sticky word, at the next call on the feeder
        pf.solve_device(d_pq, o)
    # a feeder made without the override solves the same batch
    ok = PowerFlow(f).solve(pq, full=False)
    assert (ok["status"] == 0).all()
