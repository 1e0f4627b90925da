"""The wave kernel's sequential-order plan (fpf_api.cpp: analyse_wave_lag, no
device): Dl tables whose rows do not follow the feeder tree -- which the tree
plan declines and which used to run only on the exact generic kernel -- get a
wave plan, zeroed phases included up to 256 branches (past that the generic
kernel runs them)."""
import numpy as np
import pytest

from freedm_amd import feeder as F
from lag_tables import cases, restart_cases, shuffled_blocks, wblk_cases, zeroed_cases
from test_wave_plan import _plan


@pytest.mark.parametrize("name", sorted(cases()))
def test_sequential_order_tables_get_a_wave_plan(name):
    f = cases()[name]
    p = _plan(f)
    assert p["ok"] == 1, name
    assert p["nblk"] >= 2 and p["lds"] <= 159 * 1024


@pytest.mark.parametrize("name", sorted(wblk_cases()))
def test_sequential_order_tables_get_a_wave_block_plan(name):
    f = wblk_cases()[name]
    p = _plan(f)
    assert p["ok"] == 1 and p["spw"] == 1 and p["wpb"] >= 2, (name, p)   # (wpb: the wave-block kernel's wavefronts)
    assert p["lds"] <= 159 * 1024


def test_sequential_order_tables_are_not_well_formed():
    """Every case is one the tree plan declines (well_formed 0 or a chain that
    leaves the tree): the sequential-order plan is what runs it."""
    import ctypes as C
    from freedm_amd import _lib
    from freedm_amd.engine import PowerFlow  # noqa: F401  (binding only)
    for name, f in {**cases(), **wblk_cases()}.items():
        r = _rows_chain(f.Dl)
        assert r, name


def _rows_chain(Dl):
    """True where some block row does not start at the previous row's rbus, or
    some branch's sbus has its row later (the tree plan's two conditions)."""
    row_of = {int(Dl[m, 2]): m for m in range(Dl.shape[0]) if Dl[m, 0] != 0}
    for m in range(1, Dl.shape[0]):
        if Dl[m, 0] == 0:
            continue
        s = int(Dl[m, 1])
        if Dl[m - 1, 0] != 0 and int(Dl[m - 1, 2]) != s:
            return True
        if s != 0 and row_of[s] > m:
            return True
    return False


@pytest.mark.parametrize("name", sorted(zeroed_cases()))
def test_zeroed_phases_get_a_wave_plan(name):
    """Sequential-order tables with zeroed phases (one with the rows below a
    zeroed node reading its previous-sweep V): the wave kernel's plan."""
    f = zeroed_cases()[name]
    assert _rows_chain(f.Dl), name
    p = _plan(f)
    assert p["ok"] == 1 and p["spw"] >= 1 and p["lds"] <= 159 * 1024, (name, p)


@pytest.mark.parametrize("name", sorted(restart_cases()))
def test_restart_below_zeroed_stays_generic(name):
    """A live phase below a zeroed node on this sweep's forward path (V there =
    Vr(k) - Vr(m), short of the 1e-10 bar on the small result): declined."""
    assert _plan(restart_cases()[name])["ok"] == 0


def test_zeroed_phases_past_256_branches_stay_generic():
    from lag_tables import zeroed
    f = shuffled_blocks(zeroed(F.synthetic_feeder(700, 700)), 11)
    assert _plan(f)["ok"] == 0


def test_tree_tables_keep_the_tree_plan():
    """A well-formed table's plan is unchanged (the tree plan's block count)."""
    p = _plan(F.synthetic_feeder(123, 123))
    assert p["ok"] == 1 and p["nblk"] == 13 and p["bdepth"] == 3
