"""CPU tests of the parity oracle (oracle/ref_dpf.c) and its NumPy tie-breaker.

The reference holds no golden vectors for DPF_return7, so
the oracle is "parity unpinned"; these tests pin it as far as the repository
allows: (1) the qualitative trace of Broker/output.txt (sweeps per solve,
substation row, angle pattern), (2) agreement with an independent NumPy
restatement, (3) the committed golden fixtures, (4) the reference's error
behaviour on malformed Dl tables (Armadillo bounds checks -> exceptions).
"""
import numpy as np
import pytest

from conftest import GOLDEN_NAMES, load_golden
from freedm_amd import feeder as F
from oracle import oracle as O
from oracle.np_dpf import dpf_batch_np, vvc_reduce_np


def test_demo_feeder_known_values():
    # load_system_data() feeder (load_system_data.cpp:30-55) at its default loads
    f = F.demo_feeder()
    r = O.dpf_solve(f.Dl, f.Z)
    assert r["status"] == O.REF_CONVERGED and r["iters"] == 5
    vp = r["Vpolar"]
    # substation row first: |V| = vo/bkv = 1.015, angles 0 / -120 / +120 (DPF_return7.cpp:84-89,236-238)
    assert vp[0, 0] == pytest.approx(1.015, abs=1e-15)
    assert vp[0, 1] == 0.0
    assert vp[0, 3] == pytest.approx(-120.0, abs=1e-12)
    assert vp[0, 5] == pytest.approx(120.0, abs=1e-12)
    # balanced loads and symmetric Z: the three phases have equal magnitudes
    assert np.allclose(vp[:, 0], vp[:, 2], rtol=1e-13) and np.allclose(vp[:, 0], vp[:, 4], rtol=1e-13)
    # values of the independent NumPy probe quoted in SURVEY.md section 4
    assert vp[1, 0] == pytest.approx(1.00940, abs=5e-6)
    assert vp[1, 1] == pytest.approx(-1.23165, abs=5e-6)
    ln = O.lnum(f.Dl, f.Z)
    assert ln == [8, 8, 8]
    loss, vmin, vmax = O.vvc_reduce(r["Vpolar"], r["PQb"], r["PQL"], ln)
    assert loss == pytest.approx(11.6733, abs=5e-5)
    assert vmax == 1.015 and vmin == pytest.approx(vp[1:, 0].min())


def test_output_txt_qualitative_trace():
    # Broker/output.txt (older revision): every solve of the
    # 9-node feeder converged in <= 5 sweeps with |V| monotone along each lateral.
    f = F.demo_feeder()
    pq = F.scenario_loads(f, np.arange(64))
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=4)
    assert (c["status"] == 0).all() and c["iters"].max() <= 5


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_oracle_matches_golden(name):
    g = load_golden(name)
    c = O.dpf_batch(g["Dl"], g["Z"], g["pq"], nthreads=4)
    assert (c["iters"] == g["iters"]).all()
    assert (c["status"] == g["status"]).all()
    # the oracle is deterministic: bit-identical to its own committed output
    assert np.array_equal(c["V_re"], g["V_re"]) and np.array_equal(c["V_im"], g["V_im"])
    assert np.array_equal(c["loss"], g["loss"])
    assert np.array_equal(c["vmin"], g["vmin"]) and np.array_equal(c["vmax"], g["vmax"])
    assert np.array_equal(c["Vpolar"][:, :, :4], g["Vpolar"])


@pytest.mark.parametrize("name", ["g1_demo_batch", "g2_dlnew", "g3_123bus", "g6_missing_phase"])
def test_numpy_tie_breaker(name):
    g = load_golden(name)
    n = dpf_batch_np(g["Dl"], g["Z"], g["pq"])
    assert (n["iters"] == g["iters"]).all()
    vg = g["V_re"] + 1j * g["V_im"]
    vn = n["V_re"] + 1j * n["V_im"]
    assert np.max(np.abs(vn - vg) / np.maximum(np.abs(vg), 1e-300)) < 1e-12
    loss, vmin, vmax = vvc_reduce_np(n["Vpolar"], n["PQb"], n["PQL"], list(g["lnum"]))
    assert np.allclose(loss, g["loss"], rtol=1e-9, atol=1e-9)
    assert np.allclose(vmin, g["vmin"], rtol=1e-13) and np.allclose(vmax, g["vmax"], rtol=1e-13)


def test_missing_phase_semantics():
    g = load_golden("g6_missing_phase")
    vp = g["Vpolar"]
    # nodes 6..8 carry phase B only: |Va| = |Vc| = 0, angles read -0 + ... per :232-235
    assert (vp[0, 6:9, :] == 0).all() and (vp[4, 6:9, :] == 0).all()
    assert (vp[1, 6:9, :] == 0).all() and (vp[5, 6:9, :] == 180).all()
    assert (vp[2, 6:9, :] > 0).all()


def test_nonconvergent_status():
    g = load_golden("g5_nonconv")
    assert g["status"][0] == O.REF_NONCONVERGED and g["iters"][0] == 20
    assert g["status"][1] == O.REF_CONVERGED


def _bad(Dl, Z):
    return O.dpf_solve(Dl, Z)["status"] == O.REF_BAD_INPUT


def test_bad_inputs_mirror_reference_exceptions():
    f = F.demo_feeder()
    # trailing separator: sbus(m+1) read past the end (DPF_return7.cpp:140)
    Dl = np.vstack([f.Dl, np.zeros((1, 13))])
    assert _bad(Dl, f.Z)
    # rbus beyond the V field (:115)
    Dl = f.Dl.copy(); Dl[3, 2] = 40
    assert _bad(Dl, f.Z)
    # line code beyond Z (:175)
    Dl = f.Dl.copy(); Dl[2, 3] = 9
    assert _bad(Dl, f.Z)
    # no separator row: V has Nl entries but node Nn-1 = Nl is addressed (:115,226)
    Dl = np.delete(f.Dl, 5, axis=0)
    assert _bad(Dl, f.Z)
    # fewer than 12 columns
    assert O.lib().ref_count_nodes(O._dp(np.asfortranarray(f.Dl[:, :11])), 9, 11) < 0


def test_malformed_but_valid_order_is_solved():
    # a lateral listed before its tap's row: legal for the reference (no index
    # error); its sequential semantics must be reproduced, not rejected
    f = F.demo_feeder()
    Dl = f.Dl[[0, 6, 7, 8, 5, 1, 2, 3, 4]].copy()
    Dl[4] = 0
    Dl[4, :] = 0
    r = O.dpf_solve(Dl, f.Z)
    assert r["status"] in (O.REF_CONVERGED, O.REF_NONCONVERGED)


def test_batch_matches_single_calls():
    f = F.dl_new_feeder()
    pq = F.scenario_loads(f, np.arange(5))
    c = O.dpf_batch(f.Dl, f.Z, pq, nthreads=3)
    for s in range(5):
        Dl = f.Dl.copy()
        Dl[:, 6:12] = pq[:, :, s].T
        r = O.dpf_solve(Dl, f.Z)
        assert r["iters"] == c["iters"][s]
        assert np.array_equal(r["V"].real.T, c["V_re"][:, :, s])
        assert np.array_equal(r["Vpolar"].T, c["Vpolar"][:, :, s])
