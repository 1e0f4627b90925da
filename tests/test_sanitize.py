"""Host sanitizer run (the C ABI's host code and the oracle under
-fsanitize=address,undefined).  tests/asan/Makefile compiles the library's host
sources host-only with ASan + UBSan (the gfx950 kernel objects of the regular
build are linked unsanitised: GPU sanitizers are not available) and the oracle
with gcc's; tests/asan/asan_check.cpp drives every no-device entry point
(feeder analysis, wave plan, hipRTC source generation, shard / fold, error
paths) and the oracle's solve, batch and VVC round over the golden feeders,
the synthetic 123- and 2048-bus feeders and malformed tables.  No device is
touched."""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN_NAMES, load_golden
from freedm_amd.feeder import demo_feeder, synthetic_feeder

HERE = os.path.dirname(os.path.abspath(__file__))
ASAN = os.path.join(HERE, "asan")
LIB_OBJ = os.path.join(HERE, "..", "freedm_amd", "lib", "fpf_wave.o")


def _write(path, Dl, Z):
    Dl = np.asfortranarray(Dl, dtype=np.float64)
    Z = np.asarray(Z, dtype=np.complex128)
    with open(path, "wb") as f:
        np.array([Dl.shape[0], Dl.shape[1], Z.shape[0], Z.shape[1]], dtype=np.int32).tofile(f)
        Dl.ravel(order="F").tofile(f)
        zi = np.empty(2 * Z.size)
        zi[0::2] = Z.real.ravel(order="F")
        zi[1::2] = Z.imag.ravel(order="F")
        zi.tofile(f)


@pytest.mark.skipif(not os.path.exists(LIB_OBJ), reason="the library objects are built by __graft_entry__.build()")
def test_host_code_under_asan_ubsan(tmp_path):
    r = subprocess.run(["make", "-s", "-j8", "-C", ASAN], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    files = []
    for name in GOLDEN_NAMES:
        g = load_golden(name)
        files.append(str(tmp_path / f"{name}.bin"))
        _write(files[-1], g["Dl"], g["Z"])
    for n in (123, 2048):
        f = synthetic_feeder(n, n)
        files.append(str(tmp_path / f"syn{n}.bin"))
        _write(files[-1], f.Dl, f.Z)
    d = demo_feeder()
    bad = d.Dl.copy()
    bad[3, 2] = 99                      # rbus beyond the node count: the reference's bounds check
    files.append(str(tmp_path / "bad_rbus.bin"))
    _write(files[-1], bad, d.Z)
    files.append(str(tmp_path / "no_z.bin"))
    _write(files[-1], d.Dl, np.zeros((0, 3), np.complex128))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([os.path.join(ASAN, "build", "asan_check")] + files, capture_output=True, text=True,
                       timeout=600, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "runtime error" not in out and "AddressSanitizer" not in out, out[-4000:]
    assert "asan_check ok" in out
    assert out.count("plan rc") == len(files)
