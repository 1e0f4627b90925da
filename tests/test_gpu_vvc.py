"""GPU tests of the batched VVC step-size search (fpf_vvc_line_search) against
the reference's sequential loop (VoltVarCtrl.cpp:1330-1542: two DPF_return7
calls per step, stop at the first step whose successor raises the loss)
re-enacted here with the CPU oracle."""
import numpy as np
import pytest

from freedm_amd import feeder as F
from freedm_amd import vvc

pytestmark = pytest.mark.gpu


def _candidate(ctrl, g, nodes, c, bkva=1000.0):
    """Dl_new of one step size (:1334-1372), written out independently of the library."""
    Dl = ctrl.copy()
    for x in range(3):
        col = 7 + 2 * x
        for i in range(len(nodes[x])):
            upd = g[x][i] * (bkva / 3) * c
            for r in range(ctrl.shape[0]):
                if ctrl[r, 2] == nodes[x][i]:
                    Dl[r, col] = ctrl[r, col] - upd
    return Dl


def _sequential(ctrl, Z, g, nodes, c0, m_max, ploss_orig):
    """The reference's loop, one oracle DPF per call, two per step."""
    from oracle import oracle as O
    lnum = O.lnum(ctrl, Z)

    def loss(Dl):
        r = O.dpf_solve(Dl, Z)
        assert r["status"] == 0
        return O.vvc_reduce(r["Vpolar"], r["PQb"], r["PQL"], lnum)[0]

    c = c0
    flag = True
    for m in range(m_max):
        lo = loss(_candidate(ctrl, g, nodes, c))
        c = 1.1 * c
        ln = loss(_candidate(ctrl, g, nodes, c))
        if ln > lo:
            return m, flag, lo
        if lo > ploss_orig:
            flag = False
    return -1, flag, None


@pytest.mark.parametrize("exact", [1, 0])
@pytest.mark.parametrize("which", ["demo", "123bus"])
@pytest.mark.parametrize("sign", [1.0, -1.0])
def test_line_search_matches_sequential_reference(which, exact, sign):
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    f = F.demo_feeder() if which == "demo" else F.synthetic_feeder(123, 123)
    nodes = vvc.load_nodes(f.Dl)
    rng = np.random.default_rng(7)
    g = [rng.uniform(0.2, 1.0, len(n)) * 1e-3 for n in nodes]   # a descent-like gradient
    c0 = sign * vvc.step_size0(g)
    base = O.dpf_batch(f.Dl, f.Z, np.ascontiguousarray(f.Dl[:, 6:12].T)[:, :, None], want_full=False)
    ploss_orig = float(base["loss"][0])
    m_max = 40
    pf = PowerFlow(f, exact=exact)
    r = pf.vvc_line_search(f.Dl, g, nodes, c0, 1.1, m_max, ploss_orig)
    stop, flag, lo = _sequential(f.Dl, f.Z, g, nodes, c0, m_max, ploss_orig)
    # candidates past the stop may diverge (huge steps); the reference never solves them
    assert r["first_nonconv"] == -1 or (stop >= 0 and r["first_nonconv"] > stop + 1)
    assert r["stop"] == stop and r["reverse"] == int(not flag)
    if stop >= 0:
        if exact:
            assert r["loss"][stop] == lo
        else:
            assert r["loss"][stop] == pytest.approx(lo, rel=1e-9)


def test_load_nodes_follow_the_reference_scan():
    f = F.demo_feeder()
    nodes = vvc.load_nodes(f.Dl)
    for x in range(3):
        want = [f.Dl[i, 2] for i in range(f.nl) if int(f.Dl[i, 6 + 2 * x]) != 0]
        assert list(nodes[x]) == want[:len(nodes[x])]


@pytest.mark.parametrize("which", ["demo", "dl_new", "123bus"])
def test_round_staged_search_equals_one_batch(which):
    """fpf_vvc_round solves the first 32 step sizes as one batch and the rest only
    when the stop rule has not fired among them (fpf_vvc.cpp: vvc_line_search):
    its decisions and its losses up to the stop equal the one-batch search's
    (fpf_vvc_line_search, every candidate) bit for bit -- a scenario's result does
    not depend on the batch it is solved in -- and the step sizes it did not
    solve read NaN."""
    from freedm_amd import PowerFlow
    f = {"demo": F.demo_feeder, "dl_new": F.dl_new_feeder, "123bus": lambda: F.synthetic_feeder(123, 123)}[which]()
    pf = PowerFlow(f)
    r = pf.vvc_round(f.Dl)
    full = pf.vvc_line_search(f.Dl, r["g"], r["load_nodes"], r["c0"], 1.1, 100, r["ploss_orig"])
    stop = r["stop_fwd"]
    assert stop == full["stop"] and r["reversed"] == full["reverse"]
    solved = 101 if stop < 0 or stop + 1 >= 32 else 32
    np.testing.assert_array_equal(r["loss_fwd"][:solved], full["loss"][:solved])
    assert np.isnan(r["loss_fwd"][solved:]).all()
