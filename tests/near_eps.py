"""Scenarios whose convergence decision sits on the eps threshold (test helper).

DPF_return7 stops at the first sweep whose errmx = max_p |Ib(0,p) - Ibo(p)| is
below eps = 1e-4 (Broker/src/vvc/DPF_return7.cpp:199-210).  Scaling a
scenario's loads by lambda moves every sweep's errmx continuously, so the
number of sweeps the oracle takes is a step function of lambda: bisecting
lambda to adjacent doubles gives a pair of scenarios one ulp of load apart whose
deciding errmx lies within ~1e-15 relative of eps -- the inputs on which an
implementation that sums Ib(0) in another order (the fast kernels' prefix
scans) could take a different number of sweeps than the reference.
"""
import numpy as np


def _iters(O, Dl, Z, pq_col, lam):
    D = Dl.copy()
    D[:, 6:12] = (pq_col * lam).T
    r = O.dpf_solve(D, Z)
    return r["iters"], r


def bisect_boundary(O, feeder, pq_col, lam_lo=0.05, lam_hi=1.0, max_steps=200):
    """pq_col: [6][Nl] loads of one scenario.  Returns (pq_a, pq_b, ra, rb): two
    load columns ([6][Nl]) one ulp of one load apart on either side of the load
    scale where the oracle's sweep count changes (ra, rb: the oracle results), or
    None if it does not change on [lam_lo, lam_hi]."""
    ia, _ = _iters(O, feeder.Dl, feeder.Z, pq_col, lam_lo)
    ib, _ = _iters(O, feeder.Dl, feeder.Z, pq_col, lam_hi)
    if ia == ib:
        return None
    a, b = lam_lo, lam_hi
    for _ in range(max_steps):
        m = 0.5 * (a + b)
        if m <= a or m >= b:
            break
        im, _ = _iters(O, feeder.Dl, feeder.Z, pq_col, m)
        if im == ia:
            a = m
        else:
            b = m
    # second stage, finer: at lam = a, bisect the scale (1 + t) of one mid-sized
    # load entry (its share of Ib(0) is ~1 / Nb, so an ulp of it moves errmx ~Nb
    # times less than an ulp of lam)
    col = pq_col * a
    nz = np.flatnonzero(np.abs(col) > 0)
    j = nz[np.argsort(np.abs(col.ravel()[nz]))[len(nz) // 2]]

    def at(t):
        c = col.copy().ravel()
        c[j] *= 1.0 + sgn * t
        return c.reshape(col.shape)
    for sgn in (1.0, -1.0):   # (a PV entry lowers errmx as it grows)
        t_hi = 1e-12
        while _iters(O, feeder.Dl, feeder.Z, at(t_hi), 1.0)[0] == ia and t_hi < 0.5:
            t_hi *= 4
        if _iters(O, feeder.Dl, feeder.Z, at(t_hi), 1.0)[0] != ia:
            break
    else:   # the entry cannot move the decision: keep the lam pair
        _, ra = _iters(O, feeder.Dl, feeder.Z, pq_col, a)
        _, rb = _iters(O, feeder.Dl, feeder.Z, pq_col, b)
        return pq_col * a, pq_col * b, ra, rb
    t_lo = 0.0
    for _ in range(max_steps):
        m = 0.5 * (t_lo + t_hi)
        if m <= t_lo or m >= t_hi:
            break
        if _iters(O, feeder.Dl, feeder.Z, at(m), 1.0)[0] == ia:
            t_lo = m
        else:
            t_hi = m
    ca, cb = at(t_lo), at(t_hi)
    _, ra = _iters(O, feeder.Dl, feeder.Z, ca, 1.0)
    _, rb = _iters(O, feeder.Dl, feeder.Z, cb, 1.0)
    return ca, cb, ra, rb


def deciding_margin(r, eps=1e-4):
    """min over the oracle's sweeps of |errmx - eps| / eps (the distance of the
    closest convergence decision to the threshold)."""
    t = np.asarray(r["errmx_trace"])
    return float(np.min(np.abs(t - eps)) / eps)


def near_eps_batch(O, feeder, base_pq, n_scen, lam_lo=0.05, lam_hi=1.0):
    """[6][Nl][2 k] loads: for each of the first scenarios of base_pq ([6][Nl][B])
    whose sweep count changes on [lam_lo, lam_hi], both sides of the boundary.
    Returns (pq, margins) with the oracle's deciding margins of every scenario."""
    cols, margins = [], []
    for s in range(base_pq.shape[2]):
        if len(cols) >= n_scen:
            break
        res = bisect_boundary(O, feeder, base_pq[:, :, s], lam_lo, lam_hi)
        if res is None:
            continue
        ca, cb, ra, rb = res
        for col, r in ((ca, ra), (cb, rb)):
            cols.append(col)
            margins.append(deciding_margin(r))
    return np.ascontiguousarray(np.stack(cols, axis=2)), np.array(margins)
