"""TEST INFRASTRUCTURE ONLY: ctypes wrapper over the C parity oracle
(oracle/ref_dpf.c).  Imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg -- never by the product package freedm_amd/.

"Parity unpinned" (see ref_dpf.h): the reference cannot be compiled here
(Armadillo absent) and holds no golden vectors for DPF_return7.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libfpf_oracle.so")

REF_CONVERGED, REF_NONCONVERGED, REF_BAD_INPUT = 0, 1, -2


class RefOpts(C.Structure):
    _fields_ = [("bkva", C.c_double), ("bkv", C.c_double), ("vo_kv", C.c_double),
                ("eps", C.c_double), ("mxitr", C.c_int)]


class RefOut(C.Structure):
    _fields_ = [("vpolar", C.POINTER(C.c_double)), ("pqb", C.POINTER(C.c_double)),
                ("pql", C.POINTER(C.c_double)), ("v", C.POINTER(C.c_double)),
                ("ib", C.POINTER(C.c_double)), ("il", C.POINTER(C.c_double)),
                ("iters", C.c_int), ("status", C.c_int), ("errmx", C.c_double),
                ("errmx_trace", C.POINTER(C.c_double))]


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        dp = C.POINTER(C.c_double)
        L.ref_opts_default.argtypes = [C.POINTER(RefOpts)]
        L.ref_count_nodes.argtypes = [dp, C.c_int, C.c_int]
        L.ref_check.argtypes = [dp, C.c_int, C.c_int, C.c_int, C.c_int]
        L.ref_dpf_solve.argtypes = [dp, C.c_int, C.c_int, dp, C.c_int, C.c_int,
                                    C.POINTER(RefOpts), C.POINTER(RefOut)]
        L.ref_lnum.argtypes = [dp, C.c_int, C.c_int, dp, C.c_int, C.c_int,
                               C.c_double, C.c_double, C.POINTER(C.c_int)]
        L.ref_vvc_reduce.argtypes = [dp, dp, dp, C.c_int, C.POINTER(C.c_int), dp, dp, dp]
        L.ref_dpf_batch.argtypes = [dp, C.c_int, C.c_int, dp, C.c_int, C.c_int,
                                    C.POINTER(RefOpts), C.c_int, dp,
                                    dp, dp, dp, dp, dp,
                                    C.POINTER(C.c_int), C.POINTER(C.c_byte),
                                    dp, dp, dp, C.c_int]
        L.ref_dpf_batch_ex.argtypes = [dp, C.c_int, C.c_int, dp, C.c_int, C.c_int,
                                       C.POINTER(RefOpts), C.c_int, dp,
                                       dp, dp, dp, dp, dp,
                                       C.POINTER(C.c_int), C.POINTER(C.c_byte),
                                       dp, dp, dp, dp, C.c_int]
        _lib = L
    return _lib


def _dp(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_double))


def default_opts(**kw) -> RefOpts:
    o = RefOpts()
    lib().ref_opts_default(C.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def _fortran(Dl):
    return np.asfortranarray(np.asarray(Dl, dtype=np.float64))


def _zbuf(Z):
    Z = np.asarray(Z, dtype=np.complex128)
    buf = np.zeros(max(2 * Z.size, 2))
    buf[0:2 * Z.size:2] = Z.real.ravel(order="F")
    buf[1:2 * Z.size:2] = Z.imag.ravel(order="F")
    return buf, Z.shape


def dpf_solve(Dl, Z, opts: RefOpts | None = None) -> dict:
    """One DPF_return7 call.  Returns Vpolar/PQb/PQL (nn x 6), V (nn x 3 complex,
    Vpolar row order), Ib ((nn-1) x 3), IL (nn x 3), iters, status, errmx."""
    L = lib()
    dl = _fortran(Dl)
    nl, ncols = dl.shape
    zb, zshape = _zbuf(Z)
    zb = np.ascontiguousarray(zb)
    nn = L.ref_count_nodes(_dp(dl), nl, ncols)
    if nn < 2:
        return {"status": REF_BAD_INPUT, "iters": 0}
    vp = np.zeros((nn, 6), order="F")
    pb = np.zeros((nn, 6), order="F")
    pl = np.zeros((nn, 6), order="F")
    v = np.zeros((nn, 3), dtype=np.complex128, order="F")
    ib = np.zeros((max(nn - 1, 1), 3), dtype=np.complex128, order="F")
    il = np.zeros((nn, 3), dtype=np.complex128, order="F")
    o = opts if opts is not None else default_opts()
    trace = np.full(max(o.mxitr, 1), np.nan)
    out = RefOut(_dp(vp), _dp(pb), _dp(pl), v.ctypes.data_as(C.POINTER(C.c_double)),
                 ib.ctypes.data_as(C.POINTER(C.c_double)), il.ctypes.data_as(C.POINTER(C.c_double)),
                 0, 0, 0.0, _dp(trace))
    rc = L.ref_dpf_solve(_dp(dl), nl, ncols, _dp(zb), zshape[0], zshape[1], C.byref(o), C.byref(out))
    res = {"status": rc, "iters": out.iters, "errmx": out.errmx, "errmx_trace": trace[:max(out.iters, 0)].copy()}
    if rc >= 0:
        res.update(Vpolar=np.ascontiguousarray(vp), PQb=np.ascontiguousarray(pb),
                   PQL=np.ascontiguousarray(pl), V=np.ascontiguousarray(v),
                   Ib=np.ascontiguousarray(ib), IL=np.ascontiguousarray(il))
    return res


def lnum(Dl, Z, bkva=1000.0, bkv=12.47):
    L = lib()
    dl = _fortran(Dl)
    zb, zshape = _zbuf(Z)
    zb = np.ascontiguousarray(zb)
    out = (C.c_int * 3)()
    rc = L.ref_lnum(_dp(dl), dl.shape[0], dl.shape[1], _dp(zb), zshape[0], zshape[1], bkva, bkv, out)
    if rc:
        raise ValueError("bad feeder")
    return [out[0], out[1], out[2]]


def vvc_reduce(Vpolar, PQb, PQL, lnum3):
    L = lib()
    vp, pb, pl = (np.asfortranarray(np.asarray(x, dtype=np.float64)) for x in (Vpolar, PQb, PQL))
    ln = (C.c_int * 3)(*lnum3)
    loss, vmin, vmax = C.c_double(), C.c_double(), C.c_double()
    L.ref_vvc_reduce(_dp(vp), _dp(pb), _dp(pl), vp.shape[0], ln, C.byref(loss), C.byref(vmin), C.byref(vmax))
    return loss.value, vmin.value, vmax.value


def dpf_batch(Dl, Z, pq, opts: RefOpts | None = None, nthreads: int = 1, want_full: bool = True) -> dict:
    """Batched oracle: pq is [6][Nl][B] (scenario fastest).  Outputs are
    [col][row][B] like the product C-ABI."""
    L = lib()
    dl = _fortran(Dl)
    nl, ncols = dl.shape
    zb, zshape = _zbuf(Z)
    zb = np.ascontiguousarray(zb)
    pq = np.ascontiguousarray(pq, dtype=np.float64)
    B = pq.shape[2]
    assert pq.shape[:2] == (6, nl)
    nn = L.ref_count_nodes(_dp(dl), nl, ncols)
    out = {
        "iters": np.zeros(B, dtype=np.int32), "status": np.zeros(B, dtype=np.int8),
        "loss": np.zeros(B), "vmin": np.zeros(B), "vmax": np.zeros(B), "errmx": np.zeros(B),
    }
    if want_full:
        out.update(Vpolar=np.zeros((6, nn, B)), PQb=np.zeros((6, nn, B)), PQL=np.zeros((6, nn, B)),
                   V_re=np.zeros((3, nn, B)), V_im=np.zeros((3, nn, B)))
    o = opts if opts is not None else default_opts()
    g = out.get
    rc = L.ref_dpf_batch_ex(_dp(dl), nl, ncols, _dp(zb), zshape[0], zshape[1], C.byref(o), B, _dp(pq),
                            _dp(g("Vpolar")), _dp(g("PQb")), _dp(g("PQL")), _dp(g("V_re")), _dp(g("V_im")),
                            out["iters"].ctypes.data_as(C.POINTER(C.c_int)),
                            out["status"].ctypes.data_as(C.POINTER(C.c_byte)),
                            _dp(out["loss"]), _dp(out["vmin"]), _dp(out["vmax"]), _dp(out["errmx"]), nthreads)
    out["rc"] = rc
    return out


def vvc_gradient(Dl, Z, Vpolar, beta0: float = 0.1, bkva: float = 1000.0, bkv: float = 12.47) -> dict:
    """The VVC gradient (ref_vvc.c: VoltVarCtrl.cpp:1141-1325) at a DPF result."""
    L = lib()
    L.ref_vvc_gradient.argtypes = [C.POINTER(C.c_double), C.c_int, C.c_int, C.POINTER(C.c_double), C.c_int, C.c_int,
                                   C.POINTER(C.c_double), C.c_int, C.c_double, C.c_double, C.c_double, C.c_int,
                                   C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int),
                                   C.POINTER(C.c_double)]
    dl = _fortran(Dl)
    zb, zshape = _zbuf(Z)
    zb = np.ascontiguousarray(zb)
    vp = np.asfortranarray(np.asarray(Vpolar, dtype=np.float64))
    ld = dl.shape[0]
    g = np.zeros((3, ld))
    nodes = np.zeros((3, ld))
    nload = (C.c_int * 3)()
    stats = np.zeros(4)
    rc = L.ref_vvc_gradient(_dp(dl), dl.shape[0], dl.shape[1], _dp(zb), zshape[0], zshape[1], _dp(vp), vp.shape[0],
                            bkva, bkv, beta0, ld, _dp(g), _dp(nodes), nload, _dp(stats))
    if rc:
        raise ValueError(f"ref_vvc_gradient failed ({rc})")
    n = list(nload)
    return {"g": [g[x, :n[x]].copy() for x in range(3)], "load_nodes": [nodes[x, :n[x]].copy() for x in range(3)],
            "gmin": stats[0], "gmax": stats[1], "gabs_min": stats[2], "c0": stats[3]}


def vvc_main(Dl, Z, beta0: float = 0.1, alpha: float = 1.1, m_max: int = 100, opts: RefOpts | None = None) -> dict:
    """vvc_main's numerics, sequentially as the reference (ref_vvc.c,
    VoltVarCtrl.cpp:1141-1762): base solve, gradient, step-size search, reversal."""
    L = lib()
    L.ref_vvc_main.argtypes = [C.POINTER(C.c_double), C.c_int, C.c_int, C.POINTER(C.c_double), C.c_int, C.c_int,
                               C.POINTER(RefOpts), C.c_double, C.c_double, C.c_int, C.c_int, C.POINTER(C.c_double),
                               C.POINTER(C.c_double), C.POINTER(C.c_int), C.POINTER(C.c_double),
                               C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double)]
    dl = _fortran(Dl)
    zb, zshape = _zbuf(Z)
    zb = np.ascontiguousarray(zb)
    ld = dl.shape[0]
    g = np.zeros((3, ld))
    nodes = np.zeros((3, ld))
    nload = (C.c_int * 3)()
    lf = np.full(m_max, np.nan)
    lr = np.full(m_max, np.nan)
    out = np.zeros_like(dl, order="F")
    res = np.zeros(13)
    o = opts if opts is not None else default_opts()
    rc = L.ref_vvc_main(_dp(dl), dl.shape[0], dl.shape[1], _dp(zb), zshape[0], zshape[1], C.byref(o), beta0, alpha,
                        m_max, ld, _dp(g), _dp(nodes), nload, _dp(lf), _dp(lr), _dp(out), _dp(res))
    n = list(nload)
    keys = ["ploss_orig", "vmin_orig", "vmax_orig", "c0", "stop_fwd", "stop_rev", "reversed", "sent", "ploss_after",
            "gmin", "gmax", "gabs_min", "calls"]
    r = {k: float(v) for k, v in zip(keys, res)}
    for k in ("stop_fwd", "stop_rev", "reversed", "sent", "calls"):
        r[k] = int(r[k])
    r.update(rc=rc, g=[g[x, :n[x]].copy() for x in range(3)], load_nodes=[nodes[x, :n[x]].copy() for x in range(3)],
             loss_fwd=lf, loss_rev=lr, Dl=out)
    return r
