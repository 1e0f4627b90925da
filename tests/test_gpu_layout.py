"""The scenario-major batch layout (fpf_opts.layout = FPF_LAYOUT_SCEN_MAJOR:
pq [B][6][Nl], outputs [B][col][row]).  Every kernel must give, bit for bit,
the results of the scenario-fastest layout on the same batch: the wave kernel
and the wave-block kernel read and write the layout natively (contiguous
blocks per tile / per scenario), the generic and tiled kernels run between
the host's transposes (fpf_layout.hip).  Batch sizes leave a partial last tile.
"""
import numpy as np
import pytest

from freedm_amd import feeder as F

pytestmark = pytest.mark.gpu

CASES = [(123, "auto", 0), (123, "auto", 1), (123, "generic", 1), (700, "auto", 0), (700, "auto", 1)]


@pytest.mark.parametrize("n,kernel,exact", CASES, ids=["wave", "tiled", "generic", "wblk", "generic-700"])
def test_scenario_major_equals_scenario_fastest(n, kernel, exact):
    from freedm_amd import PowerFlow
    f = F.synthetic_feeder(n, n)
    B = 45
    pq = F.scenario_loads(f, np.arange(B))
    p0 = PowerFlow(f, kernel=kernel, exact=exact)
    p1 = PowerFlow(f, kernel=kernel, exact=exact, layout=1)
    assert p0.kernel == p1.kernel
    r0 = p0.solve(pq)
    r1 = p1.solve(np.ascontiguousarray(pq.transpose(2, 0, 1)))
    assert r1["V_re"].shape == (B, 3, p1.nn) and r1["PQb"].shape == (B, 6, p1.nn)
    for k in ("iters", "status", "loss", "vmin", "vmax"):
        np.testing.assert_array_equal(r1[k], r0[k], err_msg=k)
    for k in ("V_re", "V_im", "Vpolar", "PQb", "PQL"):
        np.testing.assert_array_equal(r1[k], r0[k].transpose(2, 0, 1), err_msg=k)
    assert r1["aggregate"] == r0["aggregate"]


@pytest.mark.parametrize("n", [123, 700])
def test_scenario_major_light_outputs_on_device(n):
    """The benched path: V and the per-scenario scalars only (the wave kernels'
    light variants), device buffers, a tile-sized and a ragged batch."""
    import torch
    from freedm_amd import PowerFlow
    f = F.synthetic_feeder(n, n)
    dev = torch.device("cuda:0")
    for B in (64, 37):
        pq = F.scenario_loads(f, np.arange(B))
        res = []
        for layout, x in ((0, pq), (1, np.ascontiguousarray(pq.transpose(2, 0, 1)))):
            pf = PowerFlow(f, layout=layout)
            sh = (3, pf.nn, B) if layout == 0 else (B, 3, pf.nn)
            out = {"v_re": torch.empty(sh, dtype=torch.float64, device=dev),
                   "v_im": torch.empty(sh, dtype=torch.float64, device=dev),
                   "iters": torch.empty(B, dtype=torch.int32, device=dev),
                   "loss": torch.empty(B, dtype=torch.float64, device=dev),
                   "vmin": torch.empty(B, dtype=torch.float64, device=dev)}
            agg = torch.zeros(8, dtype=torch.float64, device=dev)
            pf.solve_device(torch.from_numpy(x).to(dev), out, agg=agg)
            torch.cuda.synchronize()
            res.append({k: v.cpu().numpy() for k, v in out.items()} | {"agg": agg.cpu().numpy()})
        a, b = res
        for k in ("iters", "loss", "vmin", "agg"):
            np.testing.assert_array_equal(b[k], a[k], err_msg=k)
        np.testing.assert_array_equal(b["v_re"], a["v_re"].transpose(2, 0, 1))
        np.testing.assert_array_equal(b["v_im"], a["v_im"].transpose(2, 0, 1))


@pytest.mark.parametrize("n", [123, 700])
def test_multi_scenario_major(n):
    """fpf_multi_solve over the scenario-major host arrays (contiguous shards),
    on the wave kernel and on the wave-block kernel."""
    from freedm_amd import MultiPowerFlow, PowerFlow
    f = F.synthetic_feeder(n, n)
    pq = np.ascontiguousarray(F.scenario_loads(f, np.arange(50)).transpose(2, 0, 1))
    r = MultiPowerFlow(f, 1, layout=1).solve(pq)
    s = PowerFlow(f, layout=1).solve(pq)
    for k in ("iters", "status", "loss", "vmin", "vmax", "V_re", "V_im", "PQb"):
        np.testing.assert_array_equal(r[k], s[k], err_msg=k)


def test_scenario_major_past_the_grid_y_limit():
    """A scenario-major batch on the exact kernels is transposed in and out
    (fpf_layout.hip); the transpose's grid y dimension (row tiles of 32) caps
    one launch at 65535 x 32 = 2 097 120 scenarios, so a longer batch goes in
    several launches.  2.2 M scenarios of the demo feeder (device buffers):
    the scenario-major results equal the scenario-fastest ones bit for bit."""
    import torch
    from freedm_amd import PowerFlow
    f = F.demo_feeder()
    dev = torch.device("cuda:0")
    B = 2_200_000
    base = torch.from_numpy(F.scenario_loads(f, np.arange(1024))).to(dev)          # [6][Nl][1024]
    ids = torch.arange(B, device=dev)
    x0 = (base[:, :, ids % 1024] * (0.9 + 0.2 * ((ids * 2654435761) % 1000).double() / 1000.0)).contiguous()
    res = []
    for layout, x in ((0, x0), (1, x0.permute(2, 0, 1).contiguous())):
        pf = PowerFlow(f, exact=1, kernel="generic", layout=layout)
        sh = (3, pf.nn, B) if layout == 0 else (B, 3, pf.nn)
        out = {"v_re": torch.empty(sh, dtype=torch.float64, device=dev),
               "iters": torch.empty(B, dtype=torch.int32, device=dev)}
        pf.solve_device(x, out)
        torch.cuda.synchronize()
        v = out["v_re"] if layout == 0 else out["v_re"].permute(1, 2, 0)
        res.append((out["iters"].cpu(), v.cpu()))
        pf.close()
        del x, out, v
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])
