"""Feeder data: the reference's bundled feeders, its on-disk formats, and the
seeded synthetic feeders the benchmark configurations need.

Dl table schema (Broker/src/vvc/load_system_data.cpp:29):
    [ln sbus rbus lcod lng ldty P1 Q1 P2 Q2 P3 Q3 QC]
ln = branch number (0 on a lateral separator row), sbus/rbus = sending/receiving
bus, lcod = line code (1-based 3x3 block of Z), lng = length, P/Q in kW/kVAr.
Z is (3*codes) x 3 complex ohms per unit length.

Everything here is host-side data preparation (numpy); nothing here solves.
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass

import numpy as np

__all__ = [
    "Feeder", "demo_feeder", "dl_new_feeder", "ieee34_z", "synthetic_feeder",
    "load_raw_ascii", "save_raw_ascii", "load_arma_bin", "save_arma_bin",
    "scenario_loads", "hosting_loads",
]

N_COLS = 13


@dataclass
class Feeder:
    """A feeder: the Dl branch table (Nl x 13, float64) and line impedances Z
    ((3*codes) x 3, complex128).  Mirrors sysdata.Dl / sysdata.Z
    (Broker/src/vvc/load_system_data.h:6-23)."""
    Dl: np.ndarray
    Z: np.ndarray
    name: str = "feeder"

    def __post_init__(self):
        self.Dl = np.ascontiguousarray(np.asarray(self.Dl, dtype=np.float64))
        self.Z = np.ascontiguousarray(np.asarray(self.Z, dtype=np.complex128))
        if self.Dl.ndim != 2 or self.Dl.shape[1] < 12:
            raise ValueError("Dl must be Nl x 13 (at least 12 columns)")
        if self.Z.ndim != 2 or self.Z.shape[1] != 3:
            raise ValueError("Z must be (3*codes) x 3")

    @property
    def nl(self) -> int:
        return self.Dl.shape[0]

    @property
    def n_nodes(self) -> int:
        """cnt_nodes of DPF_return7.cpp:26-37."""
        return int(np.count_nonzero(self.Dl[:, 0].astype(np.int64) != 0)) + 1

    @property
    def base_pq(self) -> np.ndarray:
        """Dl columns 6..11 as a [6][Nl] array (P1 Q1 P2 Q2 P3 Q3)."""
        return np.ascontiguousarray(self.Dl[:, 6:12].T)


# --------------------------------------------------------------------------- formats

def load_raw_ascii(path: str) -> np.ndarray:
    """Armadillo raw_ascii matrix (e.g. Broker/Dl_new.mat): whitespace-separated rows."""
    return np.loadtxt(path, dtype=np.float64, ndmin=2)


def save_raw_ascii(path: str, m: np.ndarray) -> None:
    """Write in Armadillo's raw_ascii style (width 22, 12 decimals, like Dl_new.mat)."""
    m = np.asarray(m, dtype=np.float64)
    with open(path, "w") as f:
        for row in m:
            f.write("".join(f"{v:22.12e}" for v in row) + "\n")


_ARMA_HDR = {np.dtype(np.float64): b"ARMA_MAT_BIN_FN008",
             np.dtype(np.complex128): b"ARMA_MAT_BIN_FC016"}


def load_arma_bin(path: str) -> np.ndarray:
    """Armadillo arma_binary matrix: header line, '<rows> <cols>' line, then
    column-major little-endian payload (e.g. Broker_s1/xx.mat, 21x1 f64)."""
    with open(path, "rb") as f:
        head = f.readline().strip()
        dims = f.readline().split()
        payload = f.read()
    dtype = {v: k for k, v in _ARMA_HDR.items()}.get(head)
    if dtype is None:
        raise ValueError(f"unsupported Armadillo binary header {head!r}")
    rows, cols = int(dims[0]), int(dims[1])
    a = np.frombuffer(payload, dtype=dtype.newbyteorder("<"), count=rows * cols)
    return a.reshape(cols, rows).T.astype(dtype)


def save_arma_bin(path: str, m: np.ndarray) -> None:
    m = np.asarray(m)
    if m.ndim == 1:
        m = m[:, None]
    dt = np.dtype(np.complex128) if np.iscomplexobj(m) else np.dtype(np.float64)
    m = m.astype(dt)
    with open(path, "wb") as f:
        f.write(_ARMA_HDR[dt] + b"\n")
        f.write(f"{m.shape[0]} {m.shape[1]}\n".encode())
        f.write(np.asfortranarray(m).astype(dt.newbyteorder("<")).tobytes(order="F"))


# --------------------------------------------------------------------------- bundled feeders

def demo_feeder() -> Feeder:
    """The 9-row / 8-branch feeder of load_system_data() (load_system_data.cpp:30-55).

    C++ integer division is reproduced: -100/3 -> -33, 220/3 -> 73, 260/3 -> 86,
    -80/3 -> -26 (then multiplied by Rpv = 1)."""
    rpv = 1.0

    def idiv(a, b):  # C++ truncating integer division
        q = abs(a) // abs(b)
        return q if (a >= 0) == (b >= 0) else -q

    rows = [
        (1, 0, 1, 2, 1, 1, 0 * rpv),
        (2, 1, 2, 1, 1, 1, 80 * rpv),
        (3, 2, 3, 1, 1, 1, idiv(-100, 3) * rpv),
        (4, 3, 4, 1, 1, 1, idiv(220, 3) * rpv),
        (5, 4, 5, 1, 1, 1, 50 * rpv),
        None,
        (6, 1, 6, 1, 1, 1, idiv(260, 3) * rpv),
        (7, 6, 7, 1, 1, 1, idiv(-80, 3) * rpv),
        (8, 7, 8, 1, 1, 1, 75 * rpv),
    ]
    Dl = np.zeros((9, N_COLS))
    for i, r in enumerate(rows):
        if r is None:
            continue
        ln, sb, rb, lc, lg, ty, p = r
        Dl[i, :6] = (ln, sb, rb, lc, lg, ty)
        Dl[i, 6] = Dl[i, 8] = Dl[i, 10] = p
    R = np.array([[2.56769666666667, 1.02707866666667, 1.02707866666667],
                  [1.02707866666667, 2.56769666666667, 1.02707866666667],
                  [1.02707866666667, 1.02707866666667, 2.56769666666667],
                  [0.8293381333333333, 0, 0],
                  [0, 0.829338133333333, 0],
                  [0, 0, 0.82933813333333]])
    X = np.array([[7.41305000000000, 2.96522000000000, 2.96522000000000],
                  [2.96522000000000, 7.41305000000000, 2.96522000000000],
                  [2.96522000000000, 2.96522000000000, 7.41305000000000],
                  [3.732021600, 0, 0],
                  [0, 3.732021600, 0],
                  [0, 0, 3.732021600]])
    return Feeder(Dl, R + 1j * X, name="load_system_data-9row")


# IEEE 34-node test feeder line configurations 300-304 (ohms per mile), the
# configurations Broker/Dl_new.mat's line codes 1-5 refer to (code 1 = 300 on
# 800-802, code 2 = 301 on 814-850, code 3 = 302 (phase A laterals), codes 4/5 =
# 303/304 (phase B laterals)); code 7 is the in-line transformer XFM-1.
_IEEE34_CFG = {
    1: [[1.3368 + 1.3343j, 0.2101 + 0.5779j, 0.2130 + 0.5015j],
        [0.2101 + 0.5779j, 1.3238 + 1.3569j, 0.2066 + 0.4591j],
        [0.2130 + 0.5015j, 0.2066 + 0.4591j, 1.3294 + 1.3471j]],
    2: [[1.9300 + 1.4115j, 0.2327 + 0.6442j, 0.2359 + 0.5691j],
        [0.2327 + 0.6442j, 1.9157 + 1.4281j, 0.2288 + 0.5238j],
        [0.2359 + 0.5691j, 0.2288 + 0.5238j, 1.9219 + 1.4209j]],
    3: [[2.7995 + 1.4855j, 0, 0], [0, 0, 0], [0, 0, 0]],
    4: [[0, 0, 0], [0, 2.7995 + 1.4855j, 0], [0, 0, 0]],
    5: [[0, 0, 0], [0, 1.9217 + 1.4212j, 0], [0, 0, 0]],
    6: [[0, 0, 0], [0, 0, 0], [0, 0, 0]],
    7: [[0.657 + 1.414j, 0, 0], [0, 0.657 + 1.414j, 0], [0, 0, 0.657 + 1.414j]],
}

# Dl_new.mat is a 24.9 kV feeder; DPF_return7 hard-codes bkv = 12.47 kV.  The
# supplied Z is re-based by (12.47/24.9)^2 so the per-unit impedances match the
# real feeder (SURVEY.md section 7 "Missing inputs": unscaled it diverges).
DL_NEW_Z_SCALE = (12.47 / 24.9) ** 2


def ieee34_z(scale: float = DL_NEW_Z_SCALE) -> np.ndarray:
    """The supplied 21x3 Z for Broker/Dl_new.mat (codes 1-7); not bundled upstream."""
    return np.vstack([np.array(_IEEE34_CFG[c], dtype=np.complex128) for c in range(1, 8)]) * scale


_DL_NEW_PATHS = [
    os.path.join(os.path.dirname(__file__), "data", "Dl_new.mat"),
]


def dl_new_feeder(path: str | None = None, scale: float = DL_NEW_Z_SCALE) -> Feeder:
    """Broker/Dl_new.mat (41 x 13, IEEE 34-node) with the supplied Z."""
    if path is None:
        for p in _DL_NEW_PATHS:
            if os.path.exists(p):
                path = p
                break
    if path is None:
        raise FileNotFoundError("Dl_new.mat not found (freedm_amd/data/Dl_new.mat)")
    return Feeder(load_raw_ascii(path), ieee34_z(scale), name="Dl_new-34node")


# --------------------------------------------------------------------------- synthetic feeders

def _splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15))
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def _u01(seed: int, *keys) -> np.ndarray:
    """Counter-based uniform [0,1): a pure function of (seed, keys...), so any
    shard of scenarios can be generated independently."""
    with np.errstate(over="ignore"):
        h = _splitmix64(np.full((), np.uint64(seed & 0xFFFFFFFFFFFFFFFF)))
        shape = np.broadcast_shapes(*[np.shape(k) for k in keys]) if keys else ()
        h = np.broadcast_to(h, shape).copy()
        for k in keys:
            h = _splitmix64(h ^ np.asarray(k, dtype=np.uint64))
    return (h >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def synthetic_feeder(n_nodes: int = 123, seed: int = 123, n_laterals: int | None = None,
                     load_kw: float | None = None, length: tuple | None = None) -> Feeder:
    """Seeded radial feeder obeying the Dl-table invariants.

    Row 0 is the substation transformer 0 -> 1 (code 2 of load_system_data's Z);
    the main chain follows; every lateral block starts after an all-zero separator
    row and taps a node whose own branch is on an earlier row.  Nodes are numbered
    1..n_nodes-1 in row order.  Line code 1 (three-phase line) with lengths
    U[0.05, 0.5].  Base loads P ~ U[0, load_kw] per phase, Q = 0.3 P.
    """
    nb = n_nodes - 1
    if n_laterals is None:
        n_laterals = max(1, round(nb / 10)) if n_nodes <= 200 else max(1, round(nb / 14))
    # calibrated (DESIGN.md "Synthetic feeders") so the base case converges in
    # 5 sweeps with Vmin ~0.96 under load_system_data's Z (codes 1 and 2)
    if load_kw is None:
        load_kw = 4.0 if n_nodes <= 200 else 0.3
    if length is None:
        length = (0.02, 0.2) if n_nodes <= 200 else (0.001, 0.01)
    rng = np.random.default_rng(seed)
    # split nb-1 non-transformer branches into a main chain + laterals
    main_len = max(2, int(round((nb - 1) * 0.35)))
    rest = nb - 1 - main_len
    cuts = np.sort(rng.choice(np.arange(1, rest), size=n_laterals - 1, replace=False)) if n_laterals > 1 else np.array([], dtype=int)
    lat_lens = np.diff(np.concatenate([[0], cuts, [rest]])).astype(int)
    rows = []
    rows.append([1, 0, 1, 2, 1.0])               # substation XMR, code 2, length 1
    node = 1
    for _ in range(main_len):
        rows.append([0, node, node + 1, 1, rng.uniform(*length)])
        node += 1
    for L in lat_lens:
        if L <= 0:
            continue
        rows.append(None)                        # separator
        tap = int(rng.integers(1, node + 1))     # any existing node >= 1
        prev = tap
        for _ in range(L):
            rows.append([0, prev, node + 1, 1, rng.uniform(*length)])
            prev = node + 1
            node += 1
    assert node == nb, (node, nb)
    Dl = np.zeros((len(rows), N_COLS))
    ln = 0
    for i, r in enumerate(rows):
        if r is None:
            continue
        ln += 1
        Dl[i, 0] = ln
        Dl[i, 1:5] = r[1:5]
        Dl[i, 5] = 1
        if i > 0:
            p = rng.uniform(0.0, load_kw, size=3)
            Dl[i, 6:12:2] = np.round(p, 3)
            Dl[i, 7:12:2] = np.round(0.3 * p, 3)
    return Feeder(Dl, demo_feeder().Z, name=f"synthetic-{n_nodes}bus-seed{seed}")


def scenario_loads(feeder: Feeder, scen_idx: np.ndarray, seed: int = 4096,
                   pv_frac: float = 0.2, pv_kw: float | None = None) -> np.ndarray:
    """Per-scenario loads [6][Nl][B] (scenario fastest) for global scenario ids.

    Config 2: per row/phase multiplier U[0.5, 1.5] on P and Q;
    a fraction pv_frac of rows gets PV with P -= U[0, pv_kw] kW per phase.
    Separator rows stay zero.  Pure function of (seed, scenario id).
    pv_kw defaults to 2/3 of the feeder's largest base per-phase load (the
    40/60 ratio of SURVEY.md 8(d))."""
    scen_idx = np.asarray(scen_idx, dtype=np.uint64)
    if pv_kw is None:
        pv_kw = (2.0 / 3.0) * float(np.max(np.abs(feeder.Dl[:, 6:12:2]))) if feeder.nl else 0.0
    nl = feeder.nl
    base = feeder.base_pq                                  # [6][Nl]
    rows = np.arange(nl, dtype=np.uint64)
    s = scen_idx[None, None, :]
    r = rows[None, :, None]
    ph = np.arange(3, dtype=np.uint64)[:, None, None]
    mult = 0.5 + _u01(seed, s, r, ph)                      # [3][Nl][B]
    has_pv = _u01(seed + 1, s, r) < pv_frac                # [1][Nl][B]
    pv = _u01(seed + 2, s, r, ph) * pv_kw                  # [3][Nl][B]
    out = np.empty((6, nl, scen_idx.size))
    live = (feeder.Dl[:, 0] != 0)[None, :, None]
    for p in range(3):
        P = base[2 * p][:, None] * mult[p] - np.where(has_pv[0], pv[p], 0.0)
        Q = base[2 * p + 1][:, None] * mult[p]
        out[2 * p] = np.where(live[0], P, 0.0)
        out[2 * p + 1] = np.where(live[0], Q, 0.0)
    return np.ascontiguousarray(out)


def hosting_loads(feeder: Feeder, scen_idx: np.ndarray, seed: int = 1 << 20,
                  pv_frac: float = 0.3, max_pen: float = 2.0) -> np.ndarray:
    """Config 4 DER hosting study: config-2 load multipliers plus PV at a random
    30 % of rows with penetration U[0, 2] x that row's base load."""
    scen_idx = np.asarray(scen_idx, dtype=np.uint64)
    nl = feeder.nl
    base = feeder.base_pq
    s = scen_idx[None, None, :]
    r = np.arange(nl, dtype=np.uint64)[None, :, None]
    ph = np.arange(3, dtype=np.uint64)[:, None, None]
    mult = 0.5 + _u01(seed, s, r, ph)
    has_pv = _u01(seed + 1, s, r) < pv_frac
    pen = _u01(seed + 2, s, r) * max_pen
    out = np.empty((6, nl, scen_idx.size))
    live = (feeder.Dl[:, 0] != 0)[:, None]
    for p in range(3):
        P = base[2 * p][:, None] * mult[p] - np.where(has_pv[0], pen[0] * base[2 * p][:, None], 0.0)
        Q = base[2 * p + 1][:, None] * mult[p]
        out[2 * p] = np.where(live, P, 0.0)
        out[2 * p + 1] = np.where(live, Q, 0.0)
    return np.ascontiguousarray(out)


# --------------------------------------------------------------------------- feeder areas (config 5)

# The master VVC's SST map on the demo feeder (Broker/src/vvc/VoltVarCtrl.cpp:442-1135):
# SST1..SST4 -> Dl rows 1..4, SST5 -> row 8, SST6 -> row 7, SST7 -> row 6; and
# the slave DGI owning each SST (Broker_s1..s3/src/vvc/VoltVarCtrl.cpp:327-395):
# s1 = SST2-4, s2 = SST1, s3 = SST5-7.
SST_ROW = {1: 1, 2: 2, 3: 3, 4: 4, 5: 8, 6: 7, 7: 6}
SST_OWNER = {1: "s2", 2: "s1", 3: "s1", 4: "s1", 5: "s3", 6: "s3", 7: "s3"}
AREA_OF_BROKER = {"s2": 0, "s1": 1, "s3": 2}   # s2 holds SST1, next to the substation: the root area


def sst_node_areas(feeder: Feeder) -> np.ndarray:
    """node_area for the multi-area solve of the demo feeder by SST ownership:
    every SST's bus (the receiving bus of its Dl row) goes to its slave's area;
    a bus without an SST (bus 1, the substation transformer's secondary) joins
    the area of its parent, else the root."""
    Dl = feeder.Dl
    nn = int((Dl[:, 0] != 0).sum()) + 1
    area = np.full(nn, -1, dtype=np.int32)
    for sst, row in SST_ROW.items():
        area[int(Dl[row, 2])] = AREA_OF_BROKER[SST_OWNER[sst]]
    par = np.zeros(nn, dtype=np.int64)
    for m in range(Dl.shape[0]):
        if Dl[m, 0] != 0:
            par[int(Dl[m, 2])] = 0 if m == 0 else int(Dl[m, 1])
    for k in range(1, nn):
        if area[k] < 0:
            area[k] = area[par[k]] if par[k] > 0 and area[par[k]] >= 0 else 0
    area[0] = 0
    return area


def subtree_node_areas(feeder: Feeder, tops) -> np.ndarray:
    """node_area with area 0 the whole feeder except the subtrees under the
    buses `tops` (area i + 1 for tops[i]; a later top nested in an earlier
    subtree takes its own part)."""
    Dl = feeder.Dl
    nn = int((Dl[:, 0] != 0).sum()) + 1
    kids = [[] for _ in range(nn)]
    for m in range(Dl.shape[0]):
        if Dl[m, 0] != 0:
            kids[0 if m == 0 else int(Dl[m, 1])].append(int(Dl[m, 2]))
    area = np.zeros(nn, dtype=np.int32)
    for i, t in enumerate(tops):
        st = [int(t)]
        while st:
            k = st.pop()
            area[k] = i + 1
            st.extend(kids[k])
    return area
