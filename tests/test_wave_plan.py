"""fpf_feeder_wave_plan (no device): the wave kernel's geometry and LDS plan
for the benched feeders, as DESIGN.md §5.0 states them."""
import ctypes as C

import numpy as np
import pytest

from freedm_amd import _lib
from freedm_amd.feeder import demo_feeder, synthetic_feeder


def _plan(f):
    L = _lib.load()
    dl = np.asfortranarray(f.Dl, dtype=np.float64)
    Z = np.asarray(f.Z, dtype=np.complex128)
    zb = np.zeros(max(2 * Z.size, 2))
    zb[0:2 * Z.size:2] = Z.real.ravel(order="F")
    zb[1:2 * Z.size:2] = Z.imag.ravel(order="F")
    o = _lib.FpfOpts()
    L.fpf_opts_default(C.byref(o))
    out = (C.c_int * 8)()
    rc = L.fpf_feeder_wave_plan(dl.ctypes.data_as(_lib._dp), dl.shape[0], dl.shape[1], zb.ctypes.data_as(_lib._dp),
                                Z.shape[0], Z.shape[1], C.byref(o), out)
    assert rc == 0
    return dict(zip(["ok", "spw", "C", "wpb", "lds", "ncomp", "nblk", "bdepth"], list(out)))


def test_123bus_plan():
    p = _plan(synthetic_feeder(123, 123))
    assert p["ok"] == 1 and (p["spw"], p["C"], p["wpb"]) == (2, 4, 8)
    # 16 scenarios x (Sld/V 6 KiB + gathered scan entries + source voltage) + the
    # compact TEMP (2 complex per slot: the reference's Z is a transposed line)
    assert p["lds"] <= 159 * 1024
    assert p["ncomp"] <= 32 and p["bdepth"] <= 4


@pytest.mark.parametrize("n", [9, 34, 65, 200, 257, 300])
def test_plan_sizes(n):
    """Every feeder of at most 256 branches gets a geometry whose L x C slots
    hold its branches; above that the wave kernel declines."""
    f = demo_feeder() if n == 9 else synthetic_feeder(n, n)
    nb = int((f.Dl[:, 0] != 0).sum())
    p = _plan(f)
    assert p["ok"] == (1 if nb <= 256 else 0)
    if p["ok"]:
        assert (64 // p["spw"]) * p["C"] >= nb and p["lds"] <= 159 * 1024
