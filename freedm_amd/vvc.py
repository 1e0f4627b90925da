"""Host-side pieces of the VVC module around the solve (Broker/src/vvc/VoltVarCtrl.cpp).

    load_nodes(Dl)           Load_a/b/c: the load buses per phase (:355-398)
    step_size0(g, ...)       c0 = beta0 / (bkva/3) / min|g| (:1316-1323)
    PowerFlow.vvc_line_search(...)  the step-size search as one batch (engine.py,
                             C ABI fpf_vvc_line_search)
"""
from __future__ import annotations

import numpy as np

BETA0 = 0.1     # min dQsst for an SST, kVAr (:1218)
ALPHA = 1.1     # step growth (:1219)
M_MAX = 100     # step-size search iterations (:1220)


def load_nodes(Dl: np.ndarray):
    """Load_a, Load_b, Load_c of vvc_main (VoltVarCtrl.cpp:355-398): the rbus of
    every row whose (int) P of that phase is nonzero, in row order.  The scan
    stops as soon as any of the node / phase counters is full (the loop guard
    of :375), which the reference relies on only implicitly."""
    Dl = np.asarray(Dl, dtype=np.float64)
    trunc = lambda x: int(x) if np.isfinite(x) and abs(x) < 2 ** 31 else 0   # (int) cast
    cnt = 1 + sum(1 for i in range(Dl.shape[0]) if trunc(Dl[i, 0]) != 0)
    nload = [sum(1 for i in range(Dl.shape[0]) if trunc(Dl[i, 6 + 2 * x]) != 0) for x in range(3)]
    out = [[], [], []]
    j = 0
    for i in range(Dl.shape[0]):
        if not (j < cnt and len(out[0]) < nload[0] and len(out[1]) < nload[1] and len(out[2]) < nload[2]):
            break
        if trunc(Dl[i, 2]) != 0:
            j += 1
        for x in range(3):
            if trunc(Dl[i, 6 + 2 * x]) != 0:
                out[x].append(float(Dl[i, 2]))
    return [np.array(v) for v in out]


def step_size0(g, bkva: float = 1000.0, beta0: float = BETA0) -> float:
    """c0 = beta0 / (bkva/3) / min over all phases of |g| (:1316-1323)."""
    gabs_min = min(float(np.min(np.abs(np.asarray(x)))) for x in g if len(x))
    return beta0 / (bkva / 3) / gabs_min


# The 21 SST set-points of the master's Gradient message (VoltVarCtrl.cpp:1504-1506):
# Q of Dl rows 1, 2, 3, 4, 6, 7, 8 (SST1..4, SST7, SST6, SST5), phase a, then b, then c
S2_ROWS = (1, 2, 3, 4, 6, 7, 8)


def s2_setpoints(Dl: np.ndarray) -> np.ndarray:
    """S2 of the Gradient message sent to the slaves (:1504-1508), 21 values (kVAr)."""
    Dl = np.asarray(Dl, dtype=np.float64)
    return np.array([Dl[r, c] for c in (7, 9, 11) for r in S2_ROWS])
