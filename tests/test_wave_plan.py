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


@pytest.mark.parametrize("n", [9, 34, 65, 200, 257, 300, 700, 1500, 2048, 2100, 3000, 4096, 4300])
def test_plan_sizes(n):
    """Every feeder of at most 256 branches gets a per-wavefront geometry whose
    L x C slots hold its branches; 257..2048 branches the wave-block kernel
    (fpf_wblk.hip: one scenario per workgroup of wpb = 2, 4, 8 wavefronts, C = 4);
    2049..4096 the paired wave-block kernel (fpf_wcoop.hip: two workgroups of 8
    wavefronts, C = 4, each holding half of the positions); above that the wave
    kernels decline."""
    f = demo_feeder() if n == 9 else synthetic_feeder(n, n)
    nb = int((f.Dl[:, 0] != 0).sum())
    p = _plan(f)
    assert p["ok"] == (1 if nb <= 4096 else 0)
    if p["ok"] and nb <= 256:
        assert (64 // p["spw"]) * p["C"] >= nb and p["lds"] <= 159 * 1024
    elif p["ok"] and nb > 2048:
        assert (p["spw"], p["C"], p["wpb"]) == (1, 4, 8)
        assert 2 * 64 * 8 * 4 >= nb and p["lds"] <= 159 * 1024
    elif p["ok"]:
        assert p["spw"] == 1 and p["C"] == 4 and p["wpb"] in (2, 4, 8)
        assert 64 * p["wpb"] * 4 >= nb > 64 * (p["wpb"] // 2) * 4
        assert p["lds"] <= 159 * 1024


def test_2048bus_plan():
    """BASELINE config 3's feeder: 8 wavefronts per scenario, the scenario's
    loads (3 x (Nl + 1) complex) plus gathered scan values and block offsets in
    one CU's LDS."""
    f = synthetic_feeder(2048, 2048)
    p = _plan(f)
    assert p["ok"] == 1 and (p["spw"], p["C"], p["wpb"]) == (1, 4, 8)
    assert 16 * 3 * (f.nl + 1) < p["lds"] <= 159 * 1024
    assert p["ncomp"] <= 510 and p["nblk"] <= 511


def test_paired_plan_zeroed_phases():
    """The paired kernel's plan (2049..4096 branches) accepts single-phase laterals
    (zeroed phases with nothing live below them) and declines a live phase below
    a zeroed one (the generic kernel runs it)."""
    import sys, os
    sys.path.insert(0, os.path.dirname(__file__))
    from test_gpu_wcoop import _single_phase_subtrees
    from test_gpu_wblk import _masked_feeder
    p = _plan(_single_phase_subtrees(3000, 3000))
    assert p["ok"] == 1 and (p["spw"], p["C"], p["wpb"]) == (1, 4, 8) and p["lds"] <= 159 * 1024
    assert _plan(_masked_feeder(3000, 3000, restart=True))["ok"] == 0


def test_paired_plan_line_codes():
    """The paired kernel keeps a slot's line code in 9 bits of a register: 70
    asymmetric codes (a 630-entry Zl table) are accepted, more than 512 codes
    declined (the generic kernel runs them)."""
    import sys, os
    sys.path.insert(0, os.path.dirname(__file__))
    from test_gpu_wcoop import _many_codes_feeder
    p = _plan(_many_codes_feeder(3000, 3000))
    assert p["ok"] == 1 and (p["spw"], p["C"], p["wpb"]) == (1, 4, 8) and p["lds"] <= 159 * 1024
    assert _plan(_many_codes_feeder(2100, 2100, ncodes=520))["ok"] == 0
