"""CPU side of the convergence guard and of the one-process multi-GPU schedule.

* tests/near_eps.py builds scenarios whose deciding errmx sits on eps: the
  oracle's sweep count differs by one across every pair it returns, and the
  closest decision is within 1e-11 relative of eps (the GPU test,
  test_gpu_guard.py, runs them through the fast kernels and the guard);
* fpf_multi_schedule (the issue order of fpf_multi_solve, no device needed):
  every device's chunk of round r is issued before any of round r - 1 is
  collected, each slot is collected before it is reused, and the chunks tile
  every device's shard -- launch-all-then-collect, so one host thread keeps
  all the devices busy.
"""
import ctypes as C

import numpy as np
import pytest

from freedm_amd import _lib
from freedm_amd import dist as D
from freedm_amd import feeder as F

from near_eps import near_eps_batch


@pytest.mark.parametrize("n,lam", [(123, (0.05, 1.0)), (123, (1.0, 3.0)), (2048, (0.05, 1.0))])
def test_near_eps_pairs_straddle_the_threshold(n, lam):
    from oracle import oracle as O
    f = F.synthetic_feeder(n, n)
    base = F.scenario_loads(f, np.arange(16))
    pq, margins = near_eps_batch(O, f, base, 6, *lam)
    assert pq.shape[2] == 6
    c = O.dpf_batch(f.Dl, f.Z, pq)
    assert (c["status"] == 0).all()
    for i in range(0, pq.shape[2], 2):
        assert c["iters"][i + 1] == c["iters"][i] + 1                     # one sweep apart
        assert np.max(np.abs(pq[:, :, i + 1] - pq[:, :, i])) <= 1e-9 * np.max(np.abs(pq[:, :, i]))
    assert margins.max() < 1e-11, margins
    # the converging side's last errmx is just below eps
    assert (c["errmx"][0::2] < 1e-4).all() and (c["errmx"][0::2] > 1e-4 * (1 - 1e-11)).all()


def _schedule(n_gpus, n_scen, chunk):
    L = _lib.load()
    n = L.fpf_multi_schedule(n_gpus, n_scen, chunk, None, 0)
    assert n >= 0
    buf = (C.c_long * (4 * max(n, 1)))()
    assert L.fpf_multi_schedule(n_gpus, n_scen, chunk, buf, n) == n
    return np.array(buf[:4 * n], dtype=np.int64).reshape(n, 4)


@pytest.mark.parametrize("n_gpus,n_scen,chunk", [(1, 10, 4), (2, 4096, 1000), (3, 100, 7), (8, 1 << 20, 65536),
                                                 (8, 5, 4), (4, 0, 16)])
def test_multi_schedule_launch_all_then_collect(n_gpus, n_scen, chunk):
    ops = _schedule(n_gpus, n_scen, chunk)
    issued, collected = [], []
    pending = {}   # (device, slot) -> chunk issued into it, not yet collected
    for pos, (kind, d, lo, hi) in enumerate(ops):
        lo_d, hi_d = D.shard_range(d, n_gpus, n_scen)
        r = (lo - lo_d) // chunk
        assert lo_d <= lo < hi <= hi_d and hi - lo <= chunk and (lo - lo_d) % chunk == 0
        if kind == 0:
            assert (d, r % 2) not in pending          # the slot was collected before reuse
            pending[(d, r % 2)] = (lo, hi)
            issued.append((pos, d, r))
        else:
            assert pending.pop((d, r % 2)) == (lo, hi)
            collected.append((pos, d, r))
    assert not pending
    # every issue of round r precedes every collect of round r - 1 (and of round r)
    for pos_c, d_c, r_c in collected:
        for pos_i, d_i, r_i in issued:
            if r_i <= r_c + 1:
                assert pos_i < pos_c
    # the chunks tile every shard
    for d in range(n_gpus):
        lo_d, hi_d = D.shard_range(d, n_gpus, n_scen)
        got = sorted((lo, hi) for kind, dd, lo, hi in ops if kind == 0 and dd == d)
        assert sum(hi - lo for lo, hi in got) == hi_d - lo_d
        assert all(got[i][1] == got[i + 1][0] for i in range(len(got) - 1))


def test_multi_schedule_bad_args():
    L = _lib.load()
    assert L.fpf_multi_schedule(0, 10, 4, None, 0) == _lib.FPF_ERR_ARG
    assert L.fpf_multi_schedule(2, 10, 0, None, 0) == _lib.FPF_ERR_ARG
