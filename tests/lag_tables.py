"""Dl tables the reference solves with its sequential semantics but whose rows
do not follow the feeder tree (DPF_return7.cpp:134-195): a block listed before
its tap's row, rows inside a block that do not chain, a branch fed from a node
whose row comes later.  Shared by tests/test_lag_plan.py (CPU: the plan) and
tests/test_gpu_lag.py (GPU: the fast kernel against the oracle)."""
import numpy as np

from freedm_amd import feeder as F


def units(Dl):
    """Block 0 (rows up to the first separator) and the [separator + block] units."""
    sep = [i for i in range(Dl.shape[0]) if Dl[i, 0] == 0]
    cut = [0] + sep + [Dl.shape[0]]
    first = Dl[:cut[1]]
    rest = [Dl[cut[i]:cut[i + 1]] for i in range(1, len(cut) - 1)]
    return first, rest


def shuffled_blocks(f, seed):
    """The feeder's lateral units in a seeded order: laterals land before their
    taps' rows (their totals are added after the tap's row; V of the tap is the
    previous sweep's)."""
    first, rest = units(f.Dl)
    order = np.random.default_rng(seed).permutation(len(rest))
    return F.Feeder(np.vstack([first] + [rest[i] for i in order]), f.Z, name=f"{f.name}-shuffled{seed}")


def reversed_blocks(f):
    """Every lateral unit after the last one that taps it... simply all units reversed."""
    first, rest = units(f.Dl)
    return F.Feeder(np.vstack([first] + rest[::-1]), f.Z, name=f"{f.name}-reversed")


def swapped_rows(f, seed, n_swaps=3):
    """Adjacent rows swapped inside blocks: the backward Ibl chain leaves the tree
    and the forward sweep reads a source before its own row."""
    Dl = f.Dl.copy()
    rng = np.random.default_rng(seed)
    cand = [i for i in range(1, Dl.shape[0] - 1) if Dl[i, 0] != 0 and Dl[i + 1, 0] != 0]
    for i in rng.choice(cand, size=min(n_swaps, len(cand)), replace=False):
        Dl[[i, i + 1]] = Dl[[i + 1, i]]
    return F.Feeder(Dl, f.Z, name=f"{f.name}-swapped{seed}")


def reordered_demo():
    f = F.demo_feeder()
    return F.Feeder(f.Dl[[0, 2, 1, 3, 4, 5, 6, 7, 8]].copy(), f.Z, name="demo-reordered")


def cases():
    f123 = F.synthetic_feeder(123, 123)
    f60 = F.synthetic_feeder(60, 60)
    return {"demo-reordered": reordered_demo(), "123-shuffled1": shuffled_blocks(f123, 1),
            "123-shuffled2": shuffled_blocks(f123, 2), "123-reversed": reversed_blocks(f123),
            "123-swapped": swapped_rows(f123, 5), "60-shuffled-swapped": swapped_rows(shuffled_blocks(f60, 3), 7),
            "200-shuffled-swapped": swapped_rows(shuffled_blocks(F.synthetic_feeder(200, 200), 4), 9)}


def wblk_cases():
    """Past 256 branches: the wave-block kernel (fpf_wblk.hip) runs the plan."""
    return {"700-shuffled-swapped": swapped_rows(shuffled_blocks(F.synthetic_feeder(700, 700), 11), 12, n_swaps=6),
            "2048-shuffled": shuffled_blocks(F.synthetic_feeder(2048, 2048), 13)}


def zeroed(f):
    """Phase c zeroed on every second lateral unit that no other unit taps (a
    two-phase line code on its rows, no phase-c load)."""
    Dl = np.array(f.Dl, copy=True)
    Z = np.vstack([f.Z, np.diag([f.Z[0, 0], f.Z[1, 1], 0])])
    code = Z.shape[0] // 3
    sep = [i for i in range(Dl.shape[0]) if Dl[i, 0] == 0] + [Dl.shape[0]]
    taps = {int(Dl[i + 1, 1]) for i in sep[:-1] if i + 1 < Dl.shape[0]}
    leaves = [u for u in range(len(sep) - 1)
              if not any(int(Dl[r, 2]) in taps for r in range(sep[u] + 1, sep[u + 1]))]
    for u in leaves[::2]:
        for r in range(sep[u] + 1, sep[u + 1]):
            Dl[r, 3] = code
            Dl[r, 10:12] = 0.0
    return F.Feeder(Dl, Z, name=f"{f.name}-zeroed")


def restart_below_zeroed(f, n_units=1):
    """Phase c zeroed on the FIRST row only of the first n_units lateral units of
    at least three rows, with no phase-c load anywhere in those units: the rows
    below keep phase c, so V there restarts from 0 at the zeroed node (V = -drop,
    the mutual coupling; DPF_return7.cpp:180-195) -- not a physical feeder, a
    table the reference solves."""
    Dl = np.array(f.Dl, copy=True)
    Z = np.vstack([f.Z, np.diag([f.Z[0, 0], f.Z[1, 1], 0])])
    code = Z.shape[0] // 3
    sep = [i for i in range(Dl.shape[0]) if Dl[i, 0] == 0] + [Dl.shape[0]]
    done = 0
    for u in range(len(sep) - 1):
        rows = list(range(sep[u] + 1, sep[u + 1]))
        if len(rows) < 3:
            continue
        Dl[rows[0], 3] = code
        Dl[rows, 10:12] = 0.0
        done += 1
        if done == n_units:
            break
    return F.Feeder(Dl, Z, name=f"{f.name}-restart")


def reordered_demo_zeroed():
    """The reordered demo table with a phase-B-only branch whose children carry
    phases A and C (no A / C load below it: V there is -drop)."""
    f = F.demo_feeder()
    Z = np.vstack([f.Z, np.diag([0, 2.0 + 6.0j, 0])])
    Dl = f.Dl[[0, 2, 1, 3, 4, 5, 6, 7, 8]].copy()
    Dl[6, 3] = 3
    Dl[7:9, [6, 7, 10, 11]] = 0
    return F.Feeder(Dl, Z, name="demo-reordered-zeroed")


def zeroed_cases():
    """Sequential-order tables with zeroed phases: the wave kernel's FULL variant
    with both general paths (GX 3)."""
    f123 = F.synthetic_feeder(123, 123)
    # (123-swapped-restart: the rows below the zeroed node read its V of the previous
    # sweep -- their row swapped ahead of its -- so the restart comes with that V,
    # exactly 0 on the phase, and no difference of path sums is formed)
    return {"123-shuffled-zeroed": shuffled_blocks(zeroed(f123), 1),
            "123-swapped-zeroed": swapped_rows(shuffled_blocks(zeroed(f123), 2), 5),
            "60-shuffled-swapped-zeroed": swapped_rows(shuffled_blocks(zeroed(F.synthetic_feeder(60, 60)), 3), 7),
            "123-swapped-restart": swapped_rows(shuffled_blocks(restart_below_zeroed(f123, 1), 1), 5)}


def restart_cases():
    """Sequential-order tables with a live phase below a zeroed node (V there
    restarts from 0): declined by the wave kernel's plan (the generic kernel runs
    them; fpf_api.cpp: analyse_wave_lag)."""
    f123 = F.synthetic_feeder(123, 123)
    return {"demo-reordered-zeroed": reordered_demo_zeroed(),
            "123-shuffled-restart": shuffled_blocks(restart_below_zeroed(f123, 1), 1),
            "60-shuffled-restart": shuffled_blocks(restart_below_zeroed(F.synthetic_feeder(60, 60), 1), 3)}

