"""Multi-GPU study inside the C ABI (fpf_multi_*, freedm_amd/csrc/fpf_multi.cpp).

CPU: the partition (fpf_multi_shard) equals freedm_amd.dist.shard_range, and
the host fold of aggregates (fpf_aggregate_fold, the combine the RCCL
all-reduce performs) equals dist.fold_aggregates -- identity included.
GPU: fpf_multi with one device gives fpf_solve_batch's results bit for bit,
and its aggregate is the fold of the per-scenario results; ragged batches
smaller than the device count leave empty shards that still join the
all-reduce (n_gpus above the box's one GPU is the driver's 8-GPU run).
"""
import ctypes as C

import numpy as np
import pytest

from freedm_amd import _lib
from freedm_amd import dist as D
from freedm_amd import feeder as F


@pytest.mark.parametrize("world", [1, 2, 3, 7, 8])
def test_shard_matches_dist(world):
    L = _lib.load()
    for n in (0, 1, 5, 8, 13, 4096, 1 << 20, 1048577):
        cover = []
        for r in range(world):
            lo, hi = C.c_long(), C.c_long()
            assert L.fpf_multi_shard(r, world, n, C.byref(lo), C.byref(hi)) == 0
            assert (lo.value, hi.value) == D.shard_range(r, world, n)
            cover.append((lo.value, hi.value))
        assert cover[0][0] == 0 and cover[-1][1] == n
        assert all(cover[i][1] == cover[i + 1][0] for i in range(world - 1))
    lo, hi = C.c_long(), C.c_long()
    assert L.fpf_multi_shard(world, world, 10, C.byref(lo), C.byref(hi)) == _lib.FPF_ERR_ARG


def test_aggregate_fold_matches_dist():
    L = _lib.load()
    rng = np.random.default_rng(7)
    rows = np.column_stack([rng.uniform(0, 1e4, 6), rng.uniform(0.9, 1.0, 6), rng.uniform(1.0, 1.1, 6),
                            rng.integers(0, 4096, (6, 5)).astype(float)])
    parts = (_lib.FpfAggregate * 6)(*[_lib.FpfAggregate(*r) for r in rows])
    out = _lib.FpfAggregate()
    L.fpf_aggregate_fold(parts, 6, C.byref(out))
    ref = D.fold_aggregates(rows)
    got = np.array([getattr(out, k) for k in D.AGG_FIELDS])
    np.testing.assert_array_equal(got[1:], ref[1:])
    assert got[0] == pytest.approx(ref[0], rel=1e-15)
    L.fpf_aggregate_fold(parts, 0, C.byref(out))
    assert (out.vmin, out.vmax, out.n_scen) == (np.inf, -np.inf, 0.0)


@pytest.mark.gpu
@pytest.mark.parametrize("name,B", [("123", 4096), ("123", 3), ("demo", 37)])
def test_multi_one_gpu_equals_single(name, B):
    from freedm_amd import MultiPowerFlow, PowerFlow
    f = F.synthetic_feeder(123, 123) if name == "123" else F.demo_feeder()
    pq = F.scenario_loads(f, np.arange(B))
    single = PowerFlow(f, device=0).solve(pq)
    m = MultiPowerFlow(f, n_gpus=1)
    r = m.solve(pq)
    for k in ("V_re", "V_im", "Vpolar", "PQb", "PQL", "iters", "status", "loss", "vmin", "vmax"):
        np.testing.assert_array_equal(r[k], single[k], err_msg=k)
    ag = r["aggregate"]
    ref = D.aggregate_results(r["status"], r["loss"], r["vmin"], r["vmax"])
    assert ag["n_scen"] == B and ag["n_conv"] == ref[3] and ag["vmin"] == ref[1] and ag["vmax"] == ref[2]
    assert ag["loss_sum"] == pytest.approx(ref[0], rel=1e-12)
    assert ag == single["aggregate"]
    m.close()


def test_multi_create_failure_reason():
    """fpf_multi_create keeps why it failed (no handle exists to carry it):
    here, more devices than the host has (none in this container)."""
    import ctypes as C
    from freedm_amd import _lib
    L = _lib.load()
    h = C.c_void_p()
    z = np.zeros(2)
    dl = np.zeros((1, 12))
    rc = L.fpf_multi_create(4096, dl.ctypes.data_as(_lib._dp), 1, 12, z.ctypes.data_as(_lib._dp), 0, 0, None, C.byref(h))
    assert rc < 0 and not h.value
    assert b"4096 devices requested" in L.fpf_multi_last_error(None)
