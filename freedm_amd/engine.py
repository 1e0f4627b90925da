"""Host-side mirror of the reference's power-flow interface over the C ABI.

    PowerFlow(feeder)            one fpf_ctx + fpf_feeder (device tables uploaded once)
      .solve(pq)                 host numpy batch  -> fpf_solve_batch
      .solve_device(pq, out)     device buffers    -> fpf_solve_batch_device (async)
    DPF_return7(Dl, Z)           the reference call (Broker/src/vvc/DPF_return7.cpp:8),
                                 a 1-scenario batch returning a VPQ record
                                 (fun_return.h:43-51); raises on non-convergence
                                 like the reference's Armadillo logic_error.

Every solve runs on the GPU through libfreedm_pf; there is no CPU path here.
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict
from dataclasses import dataclass

import numpy as np

from . import _lib
from .feeder import Feeder

__all__ = ["PowerFlow", "MultiPowerFlow", "AreaPowerFlow", "VPQ", "DPF_return7", "DPFError", "NonConvergedError",
           "ExchangeError", "FPF_EXCHANGE_FAILED"]


class DPFError(RuntimeError):
    """A libfreedm_pf error (FPF_ERR_*)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"fpf error {code}: {msg}")
        self.code = code


FPF_ERR_EXCHANGE = -6       # include/freedm_pf.h
FPF_EXCHANGE_FAILED = 3     # per-scenario status: a paired-kernel exchange gave up


class ExchangeError(DPFError):
    """A paired-kernel exchange wait gave up (FPF_ERR_EXCHANGE; feeders of
    2049..4096 branches, two workgroups per scenario): the scenarios concerned
    have status FPF_EXCHANGE_FAILED (3).  `results` holds the batch's outputs
    when the host entry raised it."""

    def __init__(self, code: int, msg: str, results: dict | None = None):
        super().__init__(code, msg)
        self.results = results


def _raise(rc: int, msg: str, results: dict | None = None):
    if rc == FPF_ERR_EXCHANGE:
        raise ExchangeError(rc, msg, results)
    raise DPFError(rc, msg)


class NonConvergedError(DPFError):
    """DPF_return7 did not converge in mxitr sweeps.  The reference throws a
    std::logic_error (size mismatch, DPF_return7.cpp:100-101,242) at this point."""


def _ptr(a) -> int | None:
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return int(a.data_ptr())      # torch tensor on the device


class _Ctx:
    _by_dev: dict = {}

    def __init__(self, device: int):
        L = _lib.load()
        h = C.c_void_p()
        rc = L.fpf_ctx_create(device, C.byref(h))
        if rc:
            raise DPFError(rc, f"fpf_ctx_create(device={device}) failed (no HIP device?)")
        self.h = h
        self.device = device

    @classmethod
    def get(cls, device: int) -> "_Ctx":
        if device not in cls._by_dev:
            cls._by_dev[device] = _Ctx(device)
        return cls._by_dev[device]

    def err(self) -> str:
        return _lib.load().fpf_last_error(self.h).decode()


@dataclass
class VPQ:
    """Result record of DPF_return7 (fun_return.h:43-51)."""
    Vpolar: np.ndarray   # Nn x 6
    PQb: np.ndarray      # Nn x 6
    PQL: np.ndarray      # Nn x 6
    Qset_a: np.ndarray   # Dl.col(7)
    Qset_b: np.ndarray   # Dl.col(9)
    Qset_c: np.ndarray   # Dl.col(11)
    V: np.ndarray        # Nn x 3 complex (not in the reference record; row order of Vpolar)
    iters: int
    loss: float
    vmin: float
    vmax: float


def _host_batch(pq, nl: int, nn: int, smaj: bool, full: bool):
    """Check a host batch's shape for the layout; allocate the host results."""
    pq = np.ascontiguousarray(pq, dtype=np.float64)
    if pq.ndim != 3 or (pq.shape[1:] if smaj else pq.shape[:2]) != (6, nl):
        raise ValueError(f"pq must be [B][6][{nl}]" if smaj else f"pq must be [6][{nl}][B]")
    B = pq.shape[0] if smaj else pq.shape[2]
    r = {"iters": np.zeros(B, np.int32), "status": np.zeros(B, np.int8), "loss": np.zeros(B),
         "vmin": np.zeros(B), "vmax": np.zeros(B), "errmx": np.zeros(B), "guard": np.zeros(B, np.int8)}
    if full:
        sh6, sh3 = ((B, 6, nn), (B, 3, nn)) if smaj else ((6, nn, B), (3, nn, B))
        r.update(Vpolar=np.zeros(sh6), PQb=np.zeros(sh6), PQL=np.zeros(sh6), V_re=np.zeros(sh3), V_im=np.zeros(sh3))
    return pq, B, r


class PowerFlow:
    """Batched DPF_return7 on one GPU for one feeder."""

    def __init__(self, feeder: Feeder, device: int = 0, kernel: str = "auto", tile: int = 0,
                 specialize: bool = True, **opts):
        L = _lib.load()
        self.feeder = feeder
        self.ctx = _Ctx.get(device)
        o = _lib.default_opts(kernel=kernel, tile=tile, specialize=int(bool(specialize)), **opts)
        self.opts = o
        dl = np.asfortranarray(feeder.Dl, dtype=np.float64)
        Z = np.asarray(feeder.Z, dtype=np.complex128)
        zbuf = np.zeros(max(2 * Z.size, 2))
        zbuf[0:2 * Z.size:2] = Z.real.ravel(order="F")
        zbuf[1:2 * Z.size:2] = Z.imag.ravel(order="F")
        h = C.c_void_p()
        rc = L.fpf_feeder_create(self.ctx.h, dl.ctypes.data_as(_lib._dp), dl.shape[0], dl.shape[1],
                                 zbuf.ctypes.data_as(_lib._dp), Z.shape[0], Z.shape[1], C.byref(o), C.byref(h))
        if rc:
            raise DPFError(rc, self.ctx.err())
        self.h = h
        info = _lib.FpfFeederInfo()
        L.fpf_feeder_get_info(h, C.byref(info))
        self.info = info.as_dict()
        self.nl, self.nn = self.info["nl"], self.info["nn"]
        self.kernel = {1: "generic", 2: "tiled", 3: "wave"}[self.info["kernel"]]
        # a hipRTC failure is not fatal (the interpreted tiled kernel runs); keep why
        self.rtc_error = self.ctx.err() if (self.kernel == "tiled" and specialize
                                            and not self.info["specialized"]) else ""

    def close(self) -> None:
        """Destroy the device feeder (fpf_feeder_destroy) now."""
        if getattr(self, "h", None):
            _lib.load().fpf_feeder_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reserve(self, n_scen: int) -> None:
        rc = _lib.load().fpf_feeder_reserve(self.h, int(n_scen))
        if rc:
            raise DPFError(rc, self.ctx.err())

    # ------------------------------------------------------------------ host batch
    def solve(self, pq: np.ndarray, full: bool = True) -> dict:
        """Solve B scenarios.  pq: [6][Nl][B] float64 (P1 Q1 P2 Q2 P3 Q3 of each
        Dl row, scenario fastest), or [B][6][Nl] for a feeder made with layout=1
        (FPF_LAYOUT_SCEN_MAJOR).  Returns per-scenario arrays ([col][row][B], or
        [B][col][row]) and the batch aggregate."""
        L = _lib.load()
        pq, B, r = _host_batch(pq, self.nl, self.nn, self.opts.layout == 1, full)
        out = _lib.FpfOutputs(_ptr(r.get("Vpolar")), _ptr(r.get("PQb")), _ptr(r.get("PQL")), _ptr(r.get("V_re")),
                              _ptr(r.get("V_im")), _ptr(r["iters"]), _ptr(r["status"]), _ptr(r["loss"]),
                              _ptr(r["vmin"]), _ptr(r["vmax"]), _ptr(r["errmx"]), _ptr(r["guard"]))
        agg = _lib.FpfAggregate()
        rc = L.fpf_solve_batch(self.h, B, pq.ctypes.data_as(_lib._dp), C.byref(out), C.byref(agg))
        if rc < 0:
            r["aggregate"] = agg.as_dict()
            _raise(rc, self.ctx.err(), r)
        r["n_nonconv"] = rc
        r["aggregate"] = agg.as_dict()
        return r

    # ------------------------------------------------------------------ device batch
    def solve_device(self, pq, out: dict, agg=None, stream=None) -> None:
        """Enqueue a solve on device buffers (torch tensors or raw pointers).
        pq: [6][Nl][B] float64 on the device; out: dict with any of
        vpolar/pqb/pql/v_re/v_im/iters/status/loss/vmin/vmax; agg: 8 float64."""
        L = _lib.load()
        B = int(pq.shape[0] if self.opts.layout == 1 else pq.shape[2])
        g = out.get
        o = _lib.FpfOutputs(_ptr(g("vpolar")), _ptr(g("pqb")), _ptr(g("pql")), _ptr(g("v_re")), _ptr(g("v_im")),
                            _ptr(g("iters")), _ptr(g("status")), _ptr(g("loss")), _ptr(g("vmin")), _ptr(g("vmax")),
                            _ptr(g("errmx")), _ptr(g("guard")))
        st = None
        if stream is not None:
            st = stream if isinstance(stream, int) else int(stream.cuda_stream)
        rc = L.fpf_solve_batch_device(self.h, B, _ptr(pq), C.byref(o), _ptr(agg), st)
        if rc < 0:
            _raise(rc, self.ctx.err())

    def check(self, stream=None) -> None:
        """fpf_feeder_check: wait for the stream, then raise ExchangeError if a
        paired-kernel launch on this feeder gave up an exchange since the last
        report (asynchronous faults of solve_device)."""
        st = None
        if stream is not None:
            st = stream if isinstance(stream, int) else int(stream.cuda_stream)
        rc = _lib.load().fpf_feeder_check(self.h, st)
        if rc < 0:
            _raise(rc, self.ctx.err())

    def bind_device(self, pq, out: dict, agg=None, stream=None):
        """Pre-bind the ctypes arguments of a device solve (and optional aggregate)
        and return (solve, aggregate) zero-argument callables -- the per-call host
        cost is then one foreign call each."""
        L = _lib.load()
        B = int(pq.shape[0] if self.opts.layout == 1 else pq.shape[2])
        g = out.get
        o = _lib.FpfOutputs(_ptr(g("vpolar")), _ptr(g("pqb")), _ptr(g("pql")), _ptr(g("v_re")), _ptr(g("v_im")),
                            _ptr(g("iters")), _ptr(g("status")), _ptr(g("loss")), _ptr(g("vmin")), _ptr(g("vmax")),
                            _ptr(g("errmx")), _ptr(g("guard")))
        st = C.c_void_p(None if stream is None else (stream if isinstance(stream, int) else int(stream.cuda_stream)))
        h, pq_p, o_ref = self.h, C.c_void_p(_ptr(pq)), C.byref(o)
        fs, fa = L.fpf_solve_batch_device, L.fpf_aggregate_device
        keep = (o,)

        def solve(agg=None):
            """One device solve; with agg (8 float64 on the device) the batch
            aggregate is produced by the same launch (specialised kernel)."""
            rc = fs(h, B, pq_p, o_ref, None if agg is None else C.c_void_p(_ptr(agg)), st)
            if rc < 0:
                _raise(rc, self.ctx.err())

        def aggregate(dst):
            rc = fa(h, B, C.c_void_p(_ptr(out["status"])), C.c_void_p(_ptr(out["loss"])), C.c_void_p(_ptr(out["vmin"])),
                    C.c_void_p(_ptr(out["vmax"])), C.c_void_p(_ptr(dst)), st)
            if rc < 0:
                raise DPFError(rc, self.ctx.err())
        solve._keep = keep
        return solve, aggregate

    def bind_aggregate(self, out: dict, agg, n_scen: int | None = None, stream=None):
        """aggregate_device with its ctypes arguments bound once: a zero-argument
        callable that enqueues the deterministic aggregate of `out` into `agg`."""
        L = _lib.load()
        B = int(out["loss"].shape[0]) if n_scen is None else int(n_scen)
        st = C.c_void_p(None if stream is None else (stream if isinstance(stream, int) else int(stream.cuda_stream)))
        args = (self.h, B, C.c_void_p(_ptr(out["status"])), C.c_void_p(_ptr(out["loss"])),
                C.c_void_p(_ptr(out["vmin"])), C.c_void_p(_ptr(out["vmax"])), C.c_void_p(_ptr(agg)), st)
        fa, ctx = L.fpf_aggregate_device, self.ctx

        def aggregate():
            rc = fa(*args)
            if rc < 0:
                raise DPFError(rc, ctx.err())
        aggregate._keep = (out, agg)
        return aggregate

    def aggregate_device(self, out: dict, agg, n_scen: int | None = None, stream=None) -> None:
        """Enqueue the deterministic batch aggregate of per-scenario device outputs."""
        L = _lib.load()
        B = int(out["loss"].shape[0]) if n_scen is None else int(n_scen)
        st = None
        if stream is not None:
            st = stream if isinstance(stream, int) else int(stream.cuda_stream)
        rc = L.fpf_aggregate_device(self.h, B, _ptr(out["status"]), _ptr(out["loss"]), _ptr(out["vmin"]),
                                    _ptr(out["vmax"]), _ptr(agg), st)
        if rc < 0:
            raise DPFError(rc, self.ctx.err())

    # ------------------------------------------------------------------ VVC step-size search
    def vvc_line_search(self, ctrl_dl: np.ndarray, g, load_nodes, c0: float, alpha: float = 1.1,
                        m_max: int = 100, ploss_orig: float = np.inf) -> dict:
        """The VVC step-size search as one batch (fpf_vvc_line_search,
        VoltVarCtrl.cpp:1316-1542; reversed search :1544-1762 = negative c0).
        g, load_nodes: three sequences (phases a, b, c) of per-load gradients
        g_vq_x and load node numbers Load_x.  Returns stop (the kept m, -1 =
        none), reverse, first_nonconv, and loss / vmin / vmax per candidate m."""
        L = _lib.load()
        ctrl = np.asfortranarray(ctrl_dl, dtype=np.float64)
        if ctrl.shape[0] != self.nl:
            raise ValueError("ctrl_dl rows differ from the feeder's")
        ld = max(1, max(len(x) for x in g))
        G = np.zeros((3, ld))
        N = np.zeros((3, ld))
        n = (C.c_int * 3)()
        for x in range(3):
            if len(g[x]) != len(load_nodes[x]):
                raise ValueError("g and load_nodes differ in length")
            G[x, :len(g[x])] = g[x]
            N[x, :len(load_nodes[x])] = load_nodes[x]
            n[x] = len(g[x])
        M = m_max + 1
        r = {"loss": np.zeros(M), "vmin": np.zeros(M), "vmax": np.zeros(M)}
        res = _lib.FpfLineSearch(0, 0, 0, 0, r["loss"].ctypes.data, r["vmin"].ctypes.data, r["vmax"].ctypes.data)
        rc = L.fpf_vvc_line_search(self.h, ctrl.ctypes.data_as(_lib._dp), ctrl.shape[0], ctrl.shape[1],
                                   G.ctypes.data_as(_lib._dp), N.ctypes.data_as(_lib._dp), n, ld, float(c0),
                                   float(alpha), int(m_max), float(ploss_orig), C.byref(res))
        if rc < 0:
            raise DPFError(rc, self.ctx.err())
        r.update(stop=res.stop, reverse=res.reverse, first_nonconv=res.first_nonconv, n_nonconv=rc)
        return r

    # ------------------------------------------------------------------ VVC gradient / round
    def _zbuf(self):
        Z = np.asarray(self.feeder.Z, dtype=np.complex128)
        zbuf = np.zeros(max(2 * Z.size, 2))
        zbuf[0:2 * Z.size:2] = Z.real.ravel(order="F")
        zbuf[1:2 * Z.size:2] = Z.imag.ravel(order="F")
        return zbuf, Z.shape

    def vvc_gradient(self, ctrl_dl: np.ndarray, beta0: float = 0.1) -> dict:
        """fpf_vvc_gradient (VoltVarCtrl.cpp:1141-1325): the loss gradient with
        respect to the SST Q injections at the control ctrl_dl."""
        L = _lib.load()
        ctrl = np.asfortranarray(ctrl_dl, dtype=np.float64)
        zbuf, zs = self._zbuf()
        ld = ctrl.shape[0]
        g, nodes, st = np.zeros((3, ld)), np.zeros((3, ld)), np.zeros(8)
        n = (C.c_int * 3)()
        rc = L.fpf_vvc_gradient(self.h, ctrl.ctypes.data_as(_lib._dp), ctrl.shape[0], ctrl.shape[1],
                                zbuf.ctypes.data_as(_lib._dp), zs[0], zs[1], float(beta0), ld,
                                g.ctypes.data_as(_lib._dp), nodes.ctypes.data_as(_lib._dp), n,
                                st.ctypes.data_as(_lib._dp))
        if rc:
            raise DPFError(rc, self.ctx.err())
        return {"g": [g[x, :n[x]].copy() for x in range(3)], "load_nodes": [nodes[x, :n[x]].copy() for x in range(3)],
                "gmin": st[0], "gmax": st[1], "gabs_min": st[2], "c0": st[3], "ploss_orig": st[4],
                "vmin_orig": st[5], "vmax_orig": st[6], "iters": int(st[7])}

    def vvc_gradient_batch(self, ctrl_dl: np.ndarray, pq: np.ndarray, beta0: float = 0.1) -> dict:
        """fpf_vvc_gradient_batch: the gradient of every scenario of pq ([6][Nl][B],
        the load columns 6..11 of ctrl_dl per scenario) as one device batch."""
        L = _lib.load()
        ctrl = np.asfortranarray(ctrl_dl, dtype=np.float64)
        pq = np.ascontiguousarray(pq, dtype=np.float64)
        if pq.ndim != 3 or pq.shape[:2] != (6, ctrl.shape[0]):
            raise ValueError(f"pq must be [6][{ctrl.shape[0]}][B]")
        B = pq.shape[2]
        zbuf, zs = self._zbuf()
        ld = ctrl.shape[0]
        g, nodes, st = np.zeros((B, 3, ld)), np.zeros((3, ld)), np.zeros((B, 8))
        gs = np.zeros(B, np.int8)
        n = (C.c_int * 3)()
        rc = L.fpf_vvc_gradient_batch(self.h, ctrl.ctypes.data_as(_lib._dp), ctrl.shape[0], ctrl.shape[1],
                                      zbuf.ctypes.data_as(_lib._dp), zs[0], zs[1], B, pq.ctypes.data_as(_lib._dp),
                                      float(beta0), ld, g.ctypes.data_as(_lib._dp), nodes.ctypes.data_as(_lib._dp), n,
                                      st.ctypes.data_as(_lib._dp), gs.ctypes.data_as(C.POINTER(C.c_int8)))
        if rc < 0:
            raise DPFError(rc, self.ctx.err())
        return {"g": [[g[s, x, :n[x]].copy() for x in range(3)] for s in range(B)],
                "load_nodes": [nodes[x, :n[x]].copy() for x in range(3)], "gstatus": gs, "n_bad": rc,
                "gmin": st[:, 0], "gmax": st[:, 1], "gabs_min": st[:, 2], "c0": st[:, 3], "ploss_orig": st[:, 4],
                "vmin_orig": st[:, 5], "vmax_orig": st[:, 6], "iters": st[:, 7].astype(int)}

    def vvc_round_batch(self, ctrl_dl: np.ndarray, pq: np.ndarray, beta0: float = 0.1, alpha: float = 1.1,
                        m_max: int = 100) -> dict:
        """fpf_vvc_round_batch: a whole VVC round (VoltVarCtrl.cpp:1141-1762) for
        every load scenario of pq ([6][Nl][B], the load columns 6..11 of ctrl_dl
        per scenario): batched gradients, all scenarios' step sizes as one batch,
        the reversed searches as another."""
        L = _lib.load()
        ctrl = np.asfortranarray(ctrl_dl, dtype=np.float64)
        pq = np.ascontiguousarray(pq, dtype=np.float64)
        if pq.ndim != 3 or pq.shape[:2] != (6, ctrl.shape[0]):
            raise ValueError(f"pq must be [6][{ctrl.shape[0]}][B]")
        B = pq.shape[2]
        zbuf, zs = self._zbuf()
        ld = ctrl.shape[0]
        g, nodes = np.zeros((B, 3, ld)), np.zeros((3, ld))
        n = (C.c_int * 3)()
        lf, lr = np.full((B, m_max + 1), np.nan), np.full((B, m_max + 1), np.nan)
        pq_out = np.zeros_like(pq)
        res = np.zeros((B, 13))
        rs = np.zeros(B, np.int8)
        rc = L.fpf_vvc_round_batch(self.h, ctrl.ctypes.data_as(_lib._dp), ctrl.shape[0], ctrl.shape[1],
                                   zbuf.ctypes.data_as(_lib._dp), zs[0], zs[1], B, pq.ctypes.data_as(_lib._dp),
                                   float(beta0), float(alpha), int(m_max), ld, g.ctypes.data_as(_lib._dp),
                                   nodes.ctypes.data_as(_lib._dp), n, lf.ctypes.data_as(_lib._dp),
                                   lr.ctypes.data_as(_lib._dp), pq_out.ctypes.data_as(_lib._dp),
                                   res.ctypes.data_as(_lib._dp), rs.ctypes.data_as(C.POINTER(C.c_int8)))
        if rc < 0:
            _raise(rc, self.ctx.err())
        keys = ["ploss_orig", "vmin_orig", "vmax_orig", "c0", "stop_fwd", "stop_rev", "reversed", "sent",
                "ploss_after", "gmin", "gmax", "gabs_min", "nonconv"]
        r = {k: res[:, i].copy() for i, k in enumerate(keys)}
        for k in ("stop_fwd", "stop_rev", "reversed", "sent", "nonconv"):
            r[k] = r[k].astype(int)
        r.update(g=[[g[s, x, :n[x]].copy() for x in range(3)] for s in range(B)],
                 load_nodes=[nodes[x, :n[x]].copy() for x in range(3)], loss_fwd=lf, loss_rev=lr, pq=pq_out,
                 rstatus=rs, n_bad=rc)
        return r

    def vvc_round(self, ctrl_dl: np.ndarray, beta0: float = 0.1, alpha: float = 1.1, m_max: int = 100) -> dict:
        """fpf_vvc_round: one VVC round of vvc_main (VoltVarCtrl.cpp:1141-1762) --
        gradient, batched step-size search, reversal -- and the control after it."""
        L = _lib.load()
        ctrl = np.asfortranarray(ctrl_dl, dtype=np.float64)
        zbuf, zs = self._zbuf()
        ld = ctrl.shape[0]
        g, nodes = np.zeros((3, ld)), np.zeros((3, ld))
        n = (C.c_int * 3)()
        lf, lr = np.full(m_max + 1, np.nan), np.full(m_max + 1, np.nan)
        out = np.zeros_like(ctrl, order="F")
        res = np.zeros(13)
        rc = L.fpf_vvc_round(self.h, ctrl.ctypes.data_as(_lib._dp), ctrl.shape[0], ctrl.shape[1],
                             zbuf.ctypes.data_as(_lib._dp), zs[0], zs[1], float(beta0), float(alpha), int(m_max), ld,
                             g.ctypes.data_as(_lib._dp), nodes.ctypes.data_as(_lib._dp), n,
                             lf.ctypes.data_as(_lib._dp), lr.ctypes.data_as(_lib._dp), out.ctypes.data_as(_lib._dp),
                             res.ctypes.data_as(_lib._dp))
        if rc < 0:
            raise DPFError(rc, self.ctx.err())
        keys = ["ploss_orig", "vmin_orig", "vmax_orig", "c0", "stop_fwd", "stop_rev", "reversed", "sent",
                "ploss_after", "gmin", "gmax", "gabs_min", "nonconv"]
        r = {k: float(v) for k, v in zip(keys, res)}
        for k in ("stop_fwd", "stop_rev", "reversed", "sent", "nonconv"):
            r[k] = int(r[k])
        r.update(g=[g[x, :n[x]].copy() for x in range(3)], load_nodes=[nodes[x, :n[x]].copy() for x in range(3)],
                 loss_fwd=lf, loss_rev=lr, Dl=out)
        return r

    # ------------------------------------------------------------------ reference call
    def dpf_return7(self, Dl: np.ndarray) -> VPQ:
        Dl = np.asarray(Dl, dtype=np.float64)
        if Dl.shape[0] != self.nl:
            raise ValueError("Dl rows differ from the feeder's")
        pq = np.ascontiguousarray(Dl[:, 6:12].T)[:, :, None]
        r = self.solve(pq, full=True)
        if r["status"][0] != 0:
            raise NonConvergedError(1, f"DPF did not converge in {int(r['iters'][0])} sweeps")
        V = (r["V_re"][:, :, 0] + 1j * r["V_im"][:, :, 0]).T
        return VPQ(Vpolar=r["Vpolar"][:, :, 0].T.copy(), PQb=r["PQb"][:, :, 0].T.copy(),
                   PQL=r["PQL"][:, :, 0].T.copy(), Qset_a=Dl[:, 7:8].copy(), Qset_b=Dl[:, 9:10].copy(),
                   Qset_c=Dl[:, 11:12].copy(), V=V, iters=int(r["iters"][0]), loss=float(r["loss"][0]),
                   vmin=float(r["vmin"][0]), vmax=float(r["vmax"][0]))


class MultiPowerFlow:
    """One process, n GPUs (fpf_multi_*): the batch is sharded contiguously over
    devices 0..n-1, every device solves its shard, and the per-device
    aggregates are combined by one RCCL all-gather inside the library, folded in
    device order (the same bits as dist.fold_aggregates)."""

    def __init__(self, feeder: Feeder, n_gpus: int = 1, kernel: str = "auto", **opts):
        L = _lib.load()
        self.feeder = feeder
        self.n_gpus = n_gpus
        o = _lib.default_opts(kernel=kernel, **opts)
        self.opts = o
        dl = np.asfortranarray(feeder.Dl, dtype=np.float64)
        Z = np.asarray(feeder.Z, dtype=np.complex128)
        zbuf = np.zeros(max(2 * Z.size, 2))
        zbuf[0:2 * Z.size:2] = Z.real.ravel(order="F")
        zbuf[1:2 * Z.size:2] = Z.imag.ravel(order="F")
        h = C.c_void_p()
        rc = L.fpf_multi_create(n_gpus, dl.ctypes.data_as(_lib._dp), dl.shape[0], dl.shape[1],
                                zbuf.ctypes.data_as(_lib._dp), Z.shape[0], Z.shape[1], C.byref(o), C.byref(h))
        if rc:
            raise DPFError(rc, L.fpf_multi_last_error(None).decode())
        self.h = h
        f0 = C.c_void_p()
        L.fpf_multi_get_feeder(h, 0, C.byref(f0))
        info = _lib.FpfFeederInfo()
        L.fpf_feeder_get_info(f0, C.byref(info))
        self.info = info.as_dict()
        self.nl, self.nn = self.info["nl"], self.info["nn"]

    def close(self) -> None:
        if getattr(self, "h", None):
            _lib.load().fpf_multi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def solve(self, pq: np.ndarray, full: bool = True) -> dict:
        """Same arguments and results as PowerFlow.solve, over all the GPUs."""
        L = _lib.load()
        pq, B, r = _host_batch(pq, self.nl, self.nn, self.opts.layout == 1, full)
        out = _lib.FpfOutputs(_ptr(r.get("Vpolar")), _ptr(r.get("PQb")), _ptr(r.get("PQL")), _ptr(r.get("V_re")),
                              _ptr(r.get("V_im")), _ptr(r["iters"]), _ptr(r["status"]), _ptr(r["loss"]),
                              _ptr(r["vmin"]), _ptr(r["vmax"]), _ptr(r["errmx"]), _ptr(r["guard"]))
        agg = _lib.FpfAggregate()
        rc = L.fpf_multi_solve(self.h, B, pq.ctypes.data_as(_lib._dp), C.byref(out), C.byref(agg))
        if rc < 0:
            raise DPFError(rc, L.fpf_multi_last_error(self.h).decode())
        r["n_nonconv"] = rc
        r["aggregate"] = agg.as_dict()
        return r


class AreaPowerFlow:
    """The multi-area solve (fpf_areas_*, BASELINE config 5): the feeder split
    into areas (node_area[k] = area of bus k), each solved as its own feeder
    fed from its boundary bus, boundary voltages and source powers exchanged
    until they settle.  eps / mxitr are the areas' inner convergence test."""

    def __init__(self, feeder: Feeder, node_area, device: int = 0, eps: float = 1e-12, mxitr: int = 200, **opts):
        L = _lib.load()
        self.feeder = feeder
        self.ctx = _Ctx.get(device)
        o = _lib.default_opts(kernel="wave", eps=eps, mxitr=mxitr, **opts)
        dl = np.asfortranarray(feeder.Dl, dtype=np.float64)
        Z = np.asarray(feeder.Z, dtype=np.complex128)
        zbuf = np.zeros(max(2 * Z.size, 2))
        zbuf[0:2 * Z.size:2] = Z.real.ravel(order="F")
        zbuf[1:2 * Z.size:2] = Z.imag.ravel(order="F")
        na = np.ascontiguousarray(node_area, dtype=np.int32)
        h = C.c_void_p()
        rc = L.fpf_areas_create(self.ctx.h, dl.ctypes.data_as(_lib._dp), dl.shape[0], dl.shape[1],
                                zbuf.ctypes.data_as(_lib._dp), Z.shape[0], Z.shape[1],
                                na.ctypes.data_as(C.POINTER(C.c_int)), na.size, C.byref(o), C.byref(h))
        if rc:
            raise DPFError(rc, f"fpf_areas_create failed: {self.ctx.err()}")
        self.h = h
        self.nl, self.nn = dl.shape[0], na.size
        n = C.c_int()
        L.fpf_areas_info(h, C.byref(n), None, None)
        nodes, parent = (C.c_int * n.value)(), (C.c_int * n.value)()
        L.fpf_areas_info(h, C.byref(n), nodes, parent)
        self.area_nodes, self.area_parent = list(nodes), list(parent)

    def close(self) -> None:
        if getattr(self, "h", None):
            _lib.load().fpf_areas_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def solve(self, pq: np.ndarray, tol: float = 1e-12, max_outer: int = 100, v_out: bool = True) -> dict:
        """v_out=False: per-scenario scalars only (no V copied back)."""
        L = _lib.load()
        pq = np.ascontiguousarray(pq, dtype=np.float64)
        if pq.ndim != 3 or pq.shape[:2] != (6, self.nl):
            raise ValueError(f"pq must be [6][{self.nl}][B]")
        B, nn = pq.shape[2], self.nn
        r = {"iters": np.zeros(B, np.int32), "status": np.zeros(B, np.int8), "loss": np.zeros(B),
             "vmin": np.zeros(B), "vmax": np.zeros(B)}
        if v_out:
            r["V_re"] = np.zeros((3, nn, B))
            r["V_im"] = np.zeros((3, nn, B))
        out = _lib.FpfOutputs(None, None, None, _ptr(r["V_re"]) if v_out else None, _ptr(r["V_im"]) if v_out else None,
                              _ptr(r["iters"]), _ptr(r["status"]), _ptr(r["loss"]), _ptr(r["vmin"]), _ptr(r["vmax"]))
        agg = _lib.FpfAggregate()
        rc = L.fpf_areas_solve(self.h, B, pq.ctypes.data_as(_lib._dp), float(tol), int(max_outer), C.byref(out),
                               C.byref(agg))
        if rc < 0:
            raise DPFError(rc, L.fpf_areas_last_error(self.h).decode())
        r["n_nonconv"] = rc
        r["aggregate"] = agg.as_dict()
        r["note"] = L.fpf_areas_last_error(self.h).decode()
        return r


_pf_cache: "OrderedDict[tuple, PowerFlow]" = OrderedDict()
PF_CACHE_SIZE = 8   # feeders kept on the device by the drop-in (least recently used evicted)


def DPF_return7(Dl: np.ndarray, Z: np.ndarray, device: int = 0, exact: bool = True) -> VPQ:
    """Drop-in for `VPQ DPF_return7(arma::mat Dl, arma::cx_mat Z)`.

    The feeder topology (columns 0..5) and Z are uploaded once and cached (at
    most PF_CACHE_SIZE feeders; the least recently used is destroyed); the
    loads (columns 6..11) travel per call.  exact=True (default) runs the
    bit-identical mode -- the reference's roundings, so a convergence test that
    lands near eps takes the reference's sweep count; exact=False is the fast
    mode (1e-10 on V)."""
    Dl = np.asarray(Dl, dtype=np.float64)
    Z = np.asarray(Z, dtype=np.complex128)
    key = (device, bool(exact), Dl.shape, Dl[:, :6].tobytes(), Z.tobytes())
    pf = _pf_cache.get(key)
    if pf is None:
        pf = PowerFlow(Feeder(Dl, Z), device=device, exact=int(bool(exact)))
        _pf_cache[key] = pf
        while len(_pf_cache) > PF_CACHE_SIZE:
            _, old = _pf_cache.popitem(last=False)
            old.close()
    else:
        _pf_cache.move_to_end(key)
    return pf.dpf_return7(Dl)
