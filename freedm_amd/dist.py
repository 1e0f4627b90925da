"""Multi-GPU sharding of a scenario study.

Scenarios are independent, so a study shards with no data-path collective:
one process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI on
ROCm, "gloo" for CPU tests), rank r solves a contiguous range of global
scenario ids, and scenario inputs are a pure function of the global id
(feeder.scenario_loads / hosting_loads), so results do not depend on the
shard.  The only exchange is the final combine of the per-GPU study
aggregates -- one all-reduce of 8 doubles:

    [loss_sum, vmin, vmax, n_conv, n_nonconv, n_over, n_under, n_scen]
     sum       min   max   sum ...

(fpf_aggregate, include/freedm_pf.h).  The reference has no counterpart: its
only "broadcast" is the per-peer UDP Gradient message of VoltVarCtrl.cpp:1497-1510,
which stays with the Broker.
"""
from __future__ import annotations

import numpy as np

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
    """Deterministic host fold of aggregate rows (the combine the all-reduce performs)."""
    rows = np.asarray(rows, dtype=np.float64).reshape(-1, 8)
    out = np.zeros(8)
    out[0] = rows[:, 0].sum()
    out[1] = rows[:, 1].min(initial=np.inf)
    out[2] = rows[:, 2].max(initial=-np.inf)
    out[3:] = rows[:, 3:].sum(axis=0)
    return out


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


def combine_aggregates(agg, group=None):
    """All-reduce one rank's 8-double aggregate (torch tensor, on the device for
    nccl/RCCL or on the CPU for gloo) in place into the study aggregate: sums for
    fields 0 and 3..7, min for vmin, max for vmax.  Two collectives of 8 and 2
    doubles -- the study's only exchange."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return agg
    mm = torch.stack([agg[1], -agg[2]])
    tot = agg.clone()
    dist.all_reduce(tot, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(mm, op=dist.ReduceOp.MIN, group=group)
    agg.copy_(tot)
    agg[1] = mm[0]
    agg[2] = -mm[1]
    return agg
