"""The topology-specialised kernel source that libfreedm_pf generates at
fpf_feeder_create compiles with hipRTC for gfx950 (no GPU needed: hipRTC is a
compiler; loading the code object is the GPU tests' job)."""
import ctypes as C
import os
import sys
import time

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def _hiprtc():
    for p in ("/opt/rocm/lib/libhiprtc.so", "libhiprtc.so"):
        try:
            return C.CDLL(p)
        except OSError:
            continue
    pytest.skip("libhiprtc not available")


OPTS = [b"--offload-arch=gfx950", b"-O3", b"-ffp-contract=off", b"-std=c++17"]


@pytest.mark.parametrize("nn,tracks", [(9, 0), (123, 0), (123, 1), (123, 2), (123, 4)])
def test_rtc_source_compiles(nn, tracks, monkeypatch):
    if tracks:
        monkeypatch.setenv("FPF_RTC_TRACKS", str(tracks))
    from rtc_dump import rtc_source
    from freedm_amd import demo_feeder, synthetic_feeder
    f = demo_feeder() if nn == 9 else synthetic_feeder(nn, nn)
    src = rtc_source(f)
    assert "fpf_rtc_tiled" in src and "__launch_bounds__(" in src
    R = _hiprtc()
    prog = C.c_void_p()
    assert R.hiprtcCreateProgram(C.byref(prog), src.encode(), b"fpf_rtc.hip", 0, None, None) == 0
    opts = (C.c_char_p * len(OPTS))(*OPTS)
    t0 = time.time()
    rc = R.hiprtcCompileProgram(prog, len(OPTS), opts)
    n = C.c_size_t()
    R.hiprtcGetProgramLogSize(prog, C.byref(n))
    log = C.create_string_buffer(n.value + 1)
    R.hiprtcGetProgramLog(prog, log)
    assert rc == 0, log.value.decode(errors="replace")[-4000:]
    R.hiprtcGetCodeSize(prog, C.byref(n))
    assert n.value > 1000
    R.hiprtcDestroyProgram(C.byref(prog))
    assert time.time() - t0 < 120
