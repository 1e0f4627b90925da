"""Multi-GPU sharding of a scenario study.

Scenarios are independent, so a study shards with no data-path collective:
one process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI on
ROCm, "gloo" for CPU tests), rank r solves a contiguous range of global
scenario ids, and scenario inputs are a pure function of the global id
(feeder.scenario_loads / hosting_loads), so results do not depend on the
shard.  The only exchange is the final combine of the per-GPU study
aggregates -- one all-gather of 8 doubles per rank, folded in rank order on
every rank (deterministic, the same fold as fold_aggregates):

    [loss_sum, vmin, vmax, n_conv, n_nonconv, n_over, n_under, n_scen]
     sum       min   max   sum ...

(fpf_aggregate, include/freedm_pf.h).  The reference has no counterpart: its
only "broadcast" is the per-peer UDP Gradient message of VoltVarCtrl.cpp:1497-1510,
which stays with the Broker.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

TRACE = bool(os.environ.get("FPF_BENCH_TRACE"))   # (diagnostics: timed_study's stages on stderr)
AGG_FIELDS = ("loss_sum", "vmin", "vmax", "n_conv", "n_nonconv", "n_over", "n_under", "n_scen")


def shard_range(rank: int, world: int, n_total: int) -> tuple[int, int]:
    """Global scenario ids [lo, hi) of `rank`: contiguous, sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world or n_total < 0:
        raise ValueError("bad shard arguments")
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def batches(lo: int, hi: int, batch: int):
    """Consecutive batches [a, b) of at most `batch` global ids covering [lo, hi)."""
    if batch < 1:
        raise ValueError("batch must be >= 1")
    for a in range(lo, hi, batch):
        yield a, min(hi, a + batch)


def fold_aggregates(rows) -> np.ndarray:
    """Deterministic host fold of aggregate rows, in row (rank) order: sums of
    fields 0 and 3..7 accumulated one row after another, min of vmin, max of
    vmax (the combine of include/freedm_pf.h: fpf_aggregate_fold)."""
    out = [0.0, np.inf, -np.inf, 0.0, 0.0, 0.0, 0.0, 0.0]
    for r in np.asarray(rows, dtype=np.float64).reshape(-1, 8).tolist():
        out[0] += r[0]
        out[1] = min(out[1], r[1])
        out[2] = max(out[2], r[2])
        for q in range(3, 8):
            out[q] += r[q]
    return np.array(out)


def aggregate_results(status, loss, vmin, vmax, lb_v: float = 0.96, ub_v: float = 1.05) -> np.ndarray:
    """The 8-double aggregate of per-scenario results (host form of dpf_aggregate_kernel)."""
    status = np.asarray(status)
    conv = status == 0
    vmin = np.asarray(vmin)[conv]
    vmax = np.asarray(vmax)[conv]
    # n_nonconv: status FPF_NONCONVERGED (1) only; FPF_EXCHANGE_FAILED (3) is neither
    return np.array([np.asarray(loss)[conv].sum(), vmin.min(initial=np.inf), vmax.max(initial=-np.inf),
                     conv.sum(), (status == 1).sum(), (vmax > ub_v).sum(), (vmin < lb_v).sum(), status.size],
                    dtype=np.float64)


def gather_aggregates(agg, group=None):
    """Every rank's 8-double aggregate as a [world, 8] tensor on every rank:
    ONE collective (all_gather; RCCL on device tensors, gloo on host ones)."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return agg.reshape(1, 8)
    if dist.get_backend(group) == "gloo":
        agg = agg.cpu()
    parts = [torch.empty_like(agg) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, agg.contiguous(), group=group)
    return torch.stack(parts)


def combine_aggregates(agg, group=None):
    """Combine one rank's 8-double aggregate (torch tensor) in place into the
    study aggregate: gather_aggregates (the study's only exchange) folded in
    rank order (fold_aggregates) -- every rank gets the same bits."""
    import torch

    rows = gather_aggregates(agg, group)
    agg.copy_(torch.from_numpy(fold_aggregates(rows.cpu().numpy())).to(agg.device))
    return agg


def timed_study(run_steps, study_aggregate, sync=None, group=None, clock=time.perf_counter, host=None):
    """The timed region of a sharded study (bench.py): the rank's solves, its
    study aggregate, then exactly one collective (gather_aggregates) and the
    rank-order fold.  The clock is read once the folded aggregate is on the host
    -- no barrier inside the region; the caller takes the max over ranks of the
    elapsed times afterwards.  host: a pinned [world * 8] float64 tensor the rows
    are copied into (one asynchronous copy, then sync(); else rows.cpu()).
    Returns (elapsed seconds, the folded aggregate)."""
    t0 = clock()
    run_steps()
    t1 = clock()
    agg = study_aggregate()
    t2 = clock()
    rows = gather_aggregates(agg, group)
    t3 = clock()
    if host is not None and rows.device.type != "cpu":
        host.copy_(rows.reshape(-1), non_blocking=True)
        if sync is not None:
            sync()   # (waits for the rank's device work and the copy)
        else:
            # (no caller-supplied sync: wait for the copy itself before reading it)
            import torch
            torch.cuda.current_stream(rows.device).synchronize()
        rh = host.numpy()
    else:
        rh = rows.cpu().numpy()   # (waits for the rank's device work)
        if sync is not None:
            sync()
    t4 = clock()
    tot = fold_aggregates(rh)
    t5 = clock()
    if TRACE:
        print(f"timed_study: steps {1e6 * (t1 - t0):.1f} us, aggregate enqueue {1e6 * (t2 - t1):.1f}, gather "
              f"{1e6 * (t3 - t2):.1f}, to host (waits) {1e6 * (t4 - t3):.1f}, fold {1e6 * (t5 - t4):.1f}",
              file=sys.stderr, flush=True)
    return t5 - t0, tot
