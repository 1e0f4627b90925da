"""Write the hipRTC source of the wave kernel libfreedm_pf builds for a feeder's
plan (no GPU needed): tools/wave_rtc_dump.py [nodes] [out] [big_batch] [full]."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from freedm_amd import _lib, synthetic_feeder, demo_feeder, dl_new_feeder  # noqa: E402


def wave_rtc_source(feeder, big_batch=1, full=0, **opts):
    L = _lib.load()
    dl = np.asfortranarray(feeder.Dl)
    Z = feeder.Z
    zb = np.zeros(2 * Z.size)
    zb[0::2] = Z.real.ravel(order="F")
    zb[1::2] = Z.imag.ravel(order="F")
    o = _lib.default_opts(**opts)
    args = (dl.ctypes.data_as(_lib._dp), dl.shape[0], dl.shape[1], zb.ctypes.data_as(_lib._dp), Z.shape[0], 3,
            C.byref(o), int(big_batch), int(full))
    n = L.fpf_feeder_wave_rtc_source(*args, None, 0)
    if n < 0:
        raise RuntimeError(f"fpf_feeder_wave_rtc_source: {n}")
    buf = C.create_string_buffer(n)
    L.fpf_feeder_wave_rtc_source(*args, buf, n)
    return buf.value.decode()


if __name__ == "__main__":
    nn = int(sys.argv[1]) if len(sys.argv) > 1 else 123
    f = {9: demo_feeder, 34: dl_new_feeder}.get(nn, lambda: synthetic_feeder(nn, nn))()
    big = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    full = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    open(sys.argv[2] if len(sys.argv) > 2 else "/tmp/wave_rtc_src.hip", "w").write(wave_rtc_source(f, big, full))
