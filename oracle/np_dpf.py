"""TEST INFRASTRUCTURE ONLY: an independent NumPy restatement of DPF_return7
(Broker/src/vvc/DPF_return7.cpp:8-263), vectorised over scenarios, used as the
tie-breaker for the C oracle (oracle/ref_dpf.c).  Written from the reference
text, not from ref_dpf.c: it uses numpy's own complex arithmetic (complex
division by Smith's method, like libgcc's __divdc3) and numpy reductions, so it
agrees with the C oracle to rounding, not bit for bit.

Semantics follow the reference literally (row loops, separator handling, the
special first branch, phase zeroing, substation-only convergence test); results
are frozen per scenario at its own converging sweep.
"""
from __future__ import annotations

import numpy as np


def dpf_batch_np(Dl, Z, pq, bkva=1000.0, bkv=12.47, vo_kv=12.47 * 1.015, eps=1e-4, mxitr=20):
    Dl = np.asarray(Dl, dtype=np.float64)
    Z = np.asarray(Z, dtype=np.complex128)
    pq = np.asarray(pq, dtype=np.float64)            # [6][Nl][B]
    nl = Dl.shape[0]
    B = pq.shape[2]
    ln, sbus, rbus, lcd, lng = Dl[:, 0], Dl[:, 1], Dl[:, 2], Dl[:, 3], Dl[:, 4]
    nn = int(np.count_nonzero(ln.astype(np.int64) != 0)) + 1

    # Sld (:46-50) -- per scenario, [Nl][3][B]
    S = (pq[0::2] + 1j * pq[1::2]).transpose(1, 0, 2) / (bkva / 3)
    Zb = 1000 * bkv ** 2 / bkva
    rz = Z.shape[0] // 3
    Zl = [Z[3 * i:3 * i + 3, :3] / Zb for i in range(rz)] or [np.zeros((3, 3), complex)]
    vo = vo_kv / bkv
    V0 = np.array([vo, -0.5 * vo + 1j * (-0.5 * np.sqrt(3)) * vo, -0.5 * vo + 1j * (0.5 * np.sqrt(3)) * vo])

    V = np.broadcast_to(V0[None, :, None], (nl, 3, B)).astype(np.complex128).copy()
    Ibo = np.zeros((3, B), complex)
    done = np.zeros(B, bool)
    iters = np.zeros(B, np.int32)
    Vf = np.zeros_like(V)
    Ibf = np.zeros((nn - 1, 3, B), complex)
    ILf = np.zeros((nn, 3, B), complex)

    def drop(m, ibrow):
        zt = Zl[int(lcd[m]) - 1]
        # lng * (Ib (1x3) . Zt (3x3)), summed over k
        return lng[m] * np.einsum("kb,ka->ab", ibrow, zt)

    for it in range(mxitr):
        IL = np.zeros((nn, 3, B), complex)
        for j in range(nl):
            if ln[j] > 0:
                r = int(rbus[j])
                v = V[r]
                with np.errstate(all="ignore"):
                    IL[r - 1] = np.where(v == 0, 0, np.conj(S[j] / np.where(v == 0, 1, v)))
        Ib = np.zeros((nn - 1, 3, B), complex)
        Ibl = np.zeros((3, B), complex)
        for m in range(nl - 1, -1, -1):
            if ln[m] == 0:
                node = int(sbus[m + 1])
                Ib[node - 1] = Ib[node - 1] + Ibl
                Ibl = np.zeros((3, B), complex)
            else:
                r = int(rbus[m])
                Ib[r - 1] = Ib[r - 1] + Ibl + IL[r - 1]
                Ibl = Ib[r - 1].copy()
        Vn = V.copy()
        Vn[1] = V0[:, None] - drop(0, Ib[0])
        for m in range(1, nl):
            if ln[m] != 0:
                zt = Zl[int(lcd[m]) - 1]
                rv = Vn[int(sbus[m])] - drop(m, Ib[int(rbus[m] - 1)])
                for p in range(3):
                    if abs(zt[p, p]) == 0:
                        rv[p] = 0
                Vn[int(rbus[m])] = rv
        errmx = np.abs(Ib[0] - Ibo).max(axis=0)
        Ibo = Ib[0].copy()
        live = ~done
        V[:, :, live] = Vn[:, :, live]
        iters[live] = it + 1
        newly = live & (errmx < eps)
        last = live & (it == mxitr - 1)
        fin = newly | last
        Vf[:, :, fin] = V[:, :, fin]
        Ibf[:, :, fin] = Ib[:, :, fin]
        ILf[:, :, fin] = IL[:, :, fin]
        done |= newly
        if done.all():
            break

    status = np.where(done, 0, 1).astype(np.int8)
    # post-processing (:222-253): output row k <-> V(k), substation first
    Vrow = Vf[:nn]
    Ibrow = np.concatenate([Ibf[:1], Ibf], axis=0)
    ILrow = np.concatenate([ILf[nn - 1:nn], ILf[:nn - 1]], axis=0)
    s3 = bkva / 3
    Sb = (s3 * Vrow) * np.conj(Ibrow)
    SL = (s3 * Vrow) * np.conj(ILrow)
    with np.errstate(all="ignore"):
        ang = (180 / np.pi) * np.arctan(Vrow.imag / Vrow.real)
    ang[~np.isfinite(ang)] = 0
    ang[:, 1] -= 180
    ang[:, 2] += 180
    Vpolar = np.empty((6, nn, B))
    PQb = np.empty((6, nn, B))
    PQL = np.empty((6, nn, B))
    for p in range(3):
        Vpolar[2 * p] = np.abs(Vrow[:, p])
        Vpolar[2 * p + 1] = ang[:, p]
        PQb[2 * p], PQb[2 * p + 1] = Sb[:, p].real, Sb[:, p].imag
        PQL[2 * p], PQL[2 * p + 1] = SL[:, p].real, SL[:, p].imag
    return {"iters": iters, "status": status, "Vpolar": Vpolar, "PQb": PQb, "PQL": PQL,
            "V_re": Vrow.real.transpose(1, 0, 2).copy(), "V_im": Vrow.imag.transpose(1, 0, 2).copy()}


def vvc_reduce_np(Vpolar, PQb, PQL, lnum):
    """loss / Vmin / Vmax per scenario from [6][nn][B] arrays (VoltVarCtrl.cpp:1152-1161,
    1201-1207; V_abc_list.cpp:7-81)."""
    nn, B = Vpolar.shape[1], Vpolar.shape[2]
    x = np.stack([PQb[2 * p, 0] - PQL[2 * p].sum(axis=0) for p in range(3)])
    loss = x.sum(axis=0)
    vmin = np.full(B, np.inf)
    vmax = np.full(B, -np.inf)
    for p in range(3):
        K = lnum[p] + 1
        vals = Vpolar[2 * p]                           # [nn][B]
        nz = vals != 0
        rank = np.cumsum(nz, axis=0)
        take = nz & (rank <= K)
        cnt = take.sum(axis=0)
        mn = np.where(take, vals, np.inf).min(axis=0)
        mx = np.where(take, vals, -np.inf).max(axis=0)
        mn = np.where(cnt < K, np.minimum(mn, 0.0), mn)   # zero padding of V_abc_list
        mx = np.where(cnt < K, np.maximum(mx, 0.0), mx)
        vmin = np.minimum(vmin, mn)
        vmax = np.maximum(vmax, mx)
    return loss, vmin, vmax
