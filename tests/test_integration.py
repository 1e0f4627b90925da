"""The Broker glue as committed source (integration/): fpf_broker.h, the C++98
core DPF_hip.cpp wraps, driven by integration/glue_check.cpp.

CPU: it compiles under the Broker's flags (-std=c++98 -pedantic -Werror,
Broker/CMakeLists.txt:55) and links against libfreedm_pf.
GPU: DPF_return7 / DPF_batch through the glue against the oracle -- exact mode,
so PQb / PQL are bit-identical (Vpolar through hypot/atan: a few ulp), the
single call equals the batch's first scenario, and a non-converged scenario
throws std::logic_error where the reference's Armadillo code throws
(DPF_return7.cpp:100-101,242).
"""
import os
import subprocess

import numpy as np
import pytest

from freedm_amd import feeder as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INTEG = os.path.join(ROOT, "integration")
BIN = os.path.join(INTEG, "build", "glue_check")


def test_glue_compiles_as_cpp98(tmp_path):
    lib = os.path.join(ROOT, "freedm_amd", "lib")
    if not os.path.exists(os.path.join(lib, "libfreedm_pf.so")):
        pytest.skip("libfreedm_pf not built")
    out = tmp_path / "glue_check"
    subprocess.run(["g++", "-std=c++98", "-pedantic", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                    "-I", INTEG, os.path.join(INTEG, "glue_check.cpp"), "-L", lib, "-lfreedm_pf", "-o", str(out)],
                   check=True, capture_output=True)
    assert out.exists()
    # the Armadillo wrapper uses nothing beyond C++98 either (no .data(), nullptr, auto, <cstdint>)
    src = open(os.path.join(INTEG, "DPF_hip.cpp")).read()
    for tok in (".data()", "nullptr", "auto ", "<cstdint>", "std::array", "emplace_back"):
        assert tok not in src, tok


def _write_input(path, f, loads, exact):
    Dl = np.asfortranarray(f.Dl, dtype=np.float64)
    Z = np.asarray(f.Z, dtype=np.complex128)
    z = np.empty(2 * Z.size)
    z[0::2] = Z.real.ravel(order="F")
    z[1::2] = Z.imag.ravel(order="F")
    with open(path, "wb") as fh:
        np.array([Dl.shape[0], Dl.shape[1], Z.shape[0], Z.shape[1], len(loads), exact], np.int32).tofile(fh)
        Dl.ravel(order="F").tofile(fh)
        z.tofile(fh)
        for ld in loads:                       # nl x 6, column-major = [6][nl]
            np.ascontiguousarray(ld).tofile(fh)


def _read_output(path):
    raw = open(path, "rb").read()
    nn, K = np.frombuffer(raw[:8], np.int32)
    off = 8
    res = []
    for _ in range(K):
        it, cv = np.frombuffer(raw[off:off + 8], np.int32)
        loss, vmin, vmax = np.frombuffer(raw[off + 8:off + 32], np.float64)
        mats = np.frombuffer(raw[off + 32:off + 32 + 3 * 48 * nn], np.float64).reshape(3, 6, nn)
        res.append({"iters": int(it), "conv": bool(cv), "loss": loss, "vmin": vmin, "vmax": vmax,
                    "Vpolar": mats[0].T, "PQb": mats[1].T, "PQL": mats[2].T})
        off += 32 + 3 * 48 * nn
    single_ok, threw = np.frombuffer(raw[off:off + 8], np.int32)
    return res, bool(single_ok), int(threw)


@pytest.mark.gpu
def test_glue_against_oracle(tmp_path):
    from oracle import oracle as O
    assert os.path.exists(BIN), "integration/build/glue_check not built (__graft_entry__.build())"
    f = F.demo_feeder()
    pq = F.scenario_loads(f, np.arange(12))             # [6][nl][K]
    pq[:, :, 7] *= 60.0                                  # diverges: the reference throws
    loads = [pq[:, :, s] for s in range(pq.shape[2])]
    _write_input(tmp_path / "in.bin", f, loads, exact=1)
    subprocess.run([BIN, str(tmp_path / "in.bin"), str(tmp_path / "out.bin"), str(tmp_path / "log.txt")],
                   check=True, timeout=120)
    res, single_ok, threw = _read_output(tmp_path / "out.bin")
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=4)
    assert single_ok
    nonconv = np.nonzero(c["status"] != 0)[0]
    assert threw == (int(nonconv[0]) if nonconv.size else -1)
    # the reference's console lines of the K single calls (DPF_return7.cpp:38,206): a
    # "Run DPF" line each, " DPF converged!" after the converged ones only
    want = []
    for s in range(len(loads)):
        want.append(f"Run DPF on {f.n_nodes} Nodes System")
        if c["status"][s] == 0:
            want.append(" DPF converged!")
    assert (tmp_path / "log.txt").read_text().splitlines() == want
    for s, r in enumerate(res):
        assert r["iters"] == c["iters"][s] and r["conv"] == (c["status"][s] == 0)
        np.testing.assert_array_equal(r["PQb"], c["PQb"][:, :, s].T)
        np.testing.assert_array_equal(r["PQL"], c["PQL"][:, :, s].T)
        np.testing.assert_allclose(r["Vpolar"], c["Vpolar"][:, :, s].T, rtol=1e-14, atol=1e-12)
        if r["conv"]:
            assert r["loss"] == c["loss"][s]
