"""Multi-area solve (BASELINE config 5; fpf_areas_*, freedm_amd/csrc/fpf_areas.cpp).

The reference's three slave DGIs own the SSTs of the demo feeder by area
(Broker_s1..s3/src/vvc/VoltVarCtrl.cpp:327-395) but never solve a power flow:
the per-area solve with boundary exchange is new, so its parity target is the
monolithic solve of the same feeder run to the same tight tolerance
(SURVEY.md 8(d) config 5): V within 1e-10 relative, loss within 1e-8, the
voltage extremes within 1e-10.  Iteration counts are not comparable (outer
iterations of the area exchange vs sweeps).
"""
import numpy as np
import pytest

from freedm_amd import feeder as F


def test_sst_areas_of_the_demo_feeder():
    f = F.demo_feeder()
    area = F.sst_node_areas(f)
    # bus: 1 2 | 3 4 5 | 6 7 8  ->  s2 (root) | s1 | s3
    assert area[1:].tolist() == [0, 0, 1, 1, 1, 2, 2, 2]
    sub = F.subtree_node_areas(F.synthetic_feeder(123, 123), [30, 60])
    assert sub[1] == 0 and set(np.unique(sub)) == {0, 1, 2}


def _tight_monolithic(f, pq):
    from oracle import oracle as O
    o = O.default_opts()
    o.eps = 1e-13
    o.mxitr = 200
    return O.dpf_batch(f.Dl, f.Z, pq, opts=o, nthreads=8)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["auto", "streams0", "streams1", "links"])
@pytest.mark.parametrize("case", ["demo_sst", "123bus_3areas", "123bus_nested"])
def test_areas_equal_monolithic(case, mode, monkeypatch):
    """Every schedule (fpf_areas.cpp): the links folded into the area solves
    (AreaHook, the default) or launched between them (FPF_AREAS_HOOKS=0), on one
    stream (the default for a chain of areas) or one stream per area (the
    default when an area has several child areas; FPF_AREAS_STREAMS=0 / 1
    forces either)."""
    from freedm_amd import AreaPowerFlow
    if mode.startswith("streams"):
        monkeypatch.setenv("FPF_AREAS_STREAMS", mode[-1])
    if mode == "links":
        monkeypatch.setenv("FPF_AREAS_HOOKS", "0")
    if case == "demo_sst":
        f = F.demo_feeder()
        node_area = F.sst_node_areas(f)
        pq = F.scenario_loads(f, np.arange(64))
    else:
        f = F.synthetic_feeder(123, 123)
        tops = [30, 60] if case == "123bus_3areas" else [20, 45, 50]
        node_area = F.subtree_node_areas(f, tops)
        pq = F.scenario_loads(f, np.arange(512))
    ap = AreaPowerFlow(f, node_area)
    assert len(ap.area_nodes) == int(node_area[1:].max()) + 1 and ap.area_parent.count(-1) == 1
    r = ap.solve(pq, tol=1e-13, max_outer=100)
    c = _tight_monolithic(f, pq)
    assert (c["status"] == 0).all() and (r["status"] == 0).all(), r["note"]
    assert r["iters"][0] >= 2
    v = r["V_re"] + 1j * r["V_im"]
    vc = c["V_re"] + 1j * c["V_im"]
    rel = float(np.max(np.abs(v - vc) / np.abs(vc)))
    assert rel <= 1e-10, (rel, r["note"])
    np.testing.assert_allclose(r["loss"], c["loss"], rtol=1e-8)
    np.testing.assert_allclose(r["vmin"], c["vmin"], rtol=1e-10)
    np.testing.assert_allclose(r["vmax"], c["vmax"], rtol=1e-10)
    ag = r["aggregate"]
    assert ag["n_conv"] == pq.shape[2] and ag["loss_sum"] == pytest.approx(r["loss"].sum(), rel=1e-12)
    ap.close()


@pytest.mark.gpu
def test_areas_schedule_and_aggregate():
    """The device-side stop (fpf_areas.cpp): scalars without V equal those with V
    bit for bit, the outer-iteration count does not depend on how many no-op
    iterations were enqueued after convergence (max_outer 100 vs the exact count),
    a max_outer below it reports every scenario non-converged after exactly
    max_outer iterations, and the aggregate counts the hosting bounds like every
    other producer."""
    from freedm_amd import AreaPowerFlow
    f = F.synthetic_feeder(123, 123)
    pq = F.scenario_loads(f, np.arange(256))
    ap = AreaPowerFlow(f, F.subtree_node_areas(f, [30, 60]))
    r = ap.solve(pq, tol=1e-12, max_outer=100)
    n = int(r["iters"][0])
    assert (r["status"] == 0).all() and n >= 3
    s = ap.solve(pq, tol=1e-12, max_outer=100, v_out=False)
    assert "V_re" not in s
    for k in ("iters", "status", "loss", "vmin", "vmax"):
        np.testing.assert_array_equal(s[k], r[k])
    e = ap.solve(pq, tol=1e-12, max_outer=n)   # no chunk beyond the last needed iteration
    for k in ("iters", "status", "loss", "vmin", "vmax", "V_re", "V_im"):
        np.testing.assert_array_equal(e[k], r[k])
    short = ap.solve(pq, tol=1e-12, max_outer=n - 1)
    assert (short["iters"] == n - 1).all() and (short["status"] != 0).all()
    assert short["aggregate"]["n_nonconv"] == pq.shape[2]
    ag = r["aggregate"]
    assert ag["n_under"] == int((r["vmin"] < 0.96).sum()) and ag["n_over"] == int((r["vmax"] > 1.05).sum())
    assert ag["n_under"] + ag["n_over"] > 0 or (r["vmin"] >= 0.96).all()
    ap.close()


@pytest.mark.gpu
def test_areas_wave_block_root_uses_link_launches():
    """An area too large for the per-wavefront kernel (a 600-bus feeder's root
    area: the wave-block kernel, which has no area hooks) runs the link-launch
    schedule (fpf_areas.cpp: hooks only when every area solves on the wave
    kernel) and still meets the monolithic solve to 1e-10."""
    from freedm_amd import AreaPowerFlow
    f = F.synthetic_feeder(600, 600)
    node_area = F.subtree_node_areas(f, [450])
    ap = AreaPowerFlow(f, node_area)
    assert len(ap.area_nodes) == 2 and max(ap.area_nodes) > 257
    pq = F.scenario_loads(f, np.arange(32))
    r = ap.solve(pq, tol=1e-13, max_outer=100)
    c = _tight_monolithic(f, pq)
    assert (c["status"] == 0).all() and (r["status"] == 0).all(), r["note"]
    v = r["V_re"] + 1j * r["V_im"]
    vc = c["V_re"] + 1j * c["V_im"]
    rel = float(np.max(np.abs(v - vc) / np.abs(vc)))
    assert rel <= 1e-10, (rel, r["note"])
    np.testing.assert_allclose(r["loss"], c["loss"], rtol=1e-8)
    ap.close()
