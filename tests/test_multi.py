"""Multi-GPU study inside the C ABI (fpf_multi_*, freedm_amd/csrc/fpf_multi.cpp).

CPU: the partition (fpf_multi_shard) equals freedm_amd.dist.shard_range, and
the host fold of aggregates (fpf_aggregate_fold: the rows fpf_multi_solve's one
RCCL all-gather brings together, folded in device order) equals
dist.fold_aggregates bit for bit -- identity included -- so the in-process and
the one-process-per-GPU forms give the same aggregate.
GPU: fpf_multi with one device gives fpf_solve_batch's results bit for bit,
its aggregate is the fold of the per-scenario results, and each solve issues
exactly one collective; ragged batches smaller than the device count leave
empty shards that still join the all-gather (n_gpus above the box's one GPU is
the driver's 8-GPU run).
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
    np.testing.assert_array_equal(got, ref)   # the same sequential sums: the same bits
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
    L = _lib.load()
    L.fpf_multi_collectives.restype = C.c_long
    c0 = L.fpf_multi_collectives()
    r = m.solve(pq)
    assert L.fpf_multi_collectives() == c0 + 1   # one all-gather per solve
    for k in ("V_re", "V_im", "Vpolar", "PQb", "PQL", "iters", "status", "loss", "vmin", "vmax"):
        np.testing.assert_array_equal(r[k], single[k], err_msg=k)
    ag = r["aggregate"]
    ref = D.aggregate_results(r["status"], r["loss"], r["vmin"], r["vmax"])
    assert ag["n_scen"] == B and ag["n_conv"] == ref[3] and ag["vmin"] == ref[1] and ag["vmax"] == ref[2]
    assert ag["loss_sum"] == pytest.approx(ref[0], rel=1e-12)
    assert ag == single["aggregate"]
    fold = D.fold_aggregates(np.array([[single["aggregate"][k] for k in D.AGG_FIELDS]]))
    np.testing.assert_array_equal(np.array([ag[k] for k in D.AGG_FIELDS]), fold)
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


@pytest.mark.parametrize("n_gpus,n_scen,chunk", [(8, 1_000_000, 65536), (3, 100_001, 7000), (2, 5, 65536), (1, 0, 16)])
def test_multi_schedule_issues_all_before_collecting(n_gpus, n_scen, chunk):
    """fpf_multi_solve's order (fpf_multi_schedule, no device needed): every
    scenario is issued once and collected once, on its shard's device; round r
    of every device is issued before round r - 1 of any device is collected
    (one host thread keeps all devices busy); a staging slot is reissued only
    after its previous chunk was collected (double buffering)."""
    import ctypes as C
    from freedm_amd import _lib
    L = _lib.load()
    n_ops = L.fpf_multi_schedule(n_gpus, n_scen, chunk, None, 0)
    assert n_ops >= 0
    buf = (C.c_long * (4 * max(n_ops, 1)))()
    assert L.fpf_multi_schedule(n_gpus, n_scen, chunk, buf, n_ops) == n_ops
    ops = np.array(buf[:4 * n_ops], dtype=np.int64).reshape(-1, 4)   # kind, device, lo, hi
    lo = np.zeros(n_gpus, np.int64)
    hi = np.zeros(n_gpus, np.int64)
    for d in range(n_gpus):
        a, b = C.c_long(), C.c_long()
        L.fpf_multi_shard(d, n_gpus, n_scen, C.byref(a), C.byref(b))
        lo[d], hi[d] = a.value, b.value
    for kind in (0, 1):
        seen = np.zeros(n_scen, np.int32)
        for k, d, a, b in ops[ops[:, 0] == kind]:
            assert lo[d] <= a < b <= hi[d] and b - a <= chunk
            seen[a:b] += 1
        assert (seen == 1).all()
    # position of each (kind, device, chunk start) in the order
    pos = {(int(k), int(d), int(a)): i for i, (k, d, a, b) in enumerate(ops)}
    rounds = {}
    for (k, d, a), i in pos.items():
        rounds[(k, d, a)] = (a - lo[d]) // chunk
    for (k, d, a), i in pos.items():
        if k != 1:
            continue
        r = rounds[(k, d, a)]
        assert pos[(0, d, a)] < i   # a chunk is collected after it was issued
        for d2 in range(n_gpus):    # ... and after round r + 1 of every device was issued
            a2 = lo[d2] + (r + 1) * chunk
            if a2 < hi[d2]:
                assert pos[(0, d2, int(a2))] < i
        # its slot (r & 1) is issued again (round r + 2) only after this collect
        a3 = lo[d] + (r + 2) * chunk
        if a3 < hi[d]:
            assert pos[(0, d, int(a3))] > i
