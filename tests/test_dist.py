"""Multi-process (world_size 2, gloo on CPU) coverage of the sharded study
(freedm_amd/dist.py): shard assignment, shard invariance of the
scenario inputs, and the one collective -- the all-gather of the study
aggregates, folded in rank order -- against the single-process aggregate of the
same scenarios.
The per-shard solves use the CPU oracle here (test infrastructure, no GPU in
this container); on the GPU box bench.py runs the same path over RCCL."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from freedm_amd import dist as D
from freedm_amd import feeder as F

N_STUDY = 96


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    from oracle import oracle as O

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    f = F.synthetic_feeder(123, 123)
    lo, hi = D.shard_range(rank, world, N_STUDY)
    rows = []
    for a, b in D.batches(lo, hi, 20):
        r = O.dpf_batch(f.Dl, f.Z, F.hosting_loads(f, np.arange(a, b)), nthreads=2, want_full=False)
        rows.append(D.aggregate_results(r["status"], r["loss"], r["vmin"], r["vmax"]))
    agg = torch.from_numpy(D.fold_aggregates(rows))
    D.combine_aggregates(agg)
    np.save(os.path.join(out_dir, f"agg{rank}.npy"), agg.numpy())
    dist.destroy_process_group()


def test_shard_range_partitions():
    for n in (0, 1, 7, 96, 1 << 20):
        for world in (1, 2, 3, 8):
            parts = [D.shard_range(r, world, n) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1
    assert list(D.batches(5, 17, 5)) == [(5, 10), (10, 15), (15, 17)]
    with pytest.raises(ValueError):
        D.shard_range(2, 2, 10)


def test_inputs_are_shard_invariant():
    f = F.synthetic_feeder(123, 123)
    full = F.hosting_loads(f, np.arange(N_STUDY))
    lo, hi = D.shard_range(1, 2, N_STUDY)
    np.testing.assert_array_equal(F.hosting_loads(f, np.arange(lo, hi)), full[:, :, lo:hi])


def test_world2_gloo_study_aggregate():
    from oracle import oracle as O
    f = F.synthetic_feeder(123, 123)
    r = O.dpf_batch(f.Dl, f.Z, F.hosting_loads(f, np.arange(N_STUDY)), nthreads=4, want_full=False)
    ref = D.aggregate_results(r["status"], r["loss"], r["vmin"], r["vmax"])
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_rank_main, args=(2, _free_port(), d), nprocs=2, join=True, start_method="spawn")
        got = [np.load(os.path.join(d, f"agg{k}.npy")) for k in range(2)]
    for g in got:   # every rank holds the study aggregate
        np.testing.assert_array_equal(g[1:], ref[1:])
        assert g[0] == pytest.approx(ref[0], rel=1e-13)
    assert got[0][7] == N_STUDY and got[0][3] + got[0][4] == N_STUDY


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_rank_launch_specs():
    """`bench.py --gpus 8` without a launcher starts 8 rank processes itself: the
    same script and arguments, RANK = LOCAL_RANK = r (cuda:r), WORLD_SIZE 8, one
    rendezvous on 127.0.0.1 (no device touched by the parent)."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    specs = bench.rank_launch_specs(8, argv, 29555, base_env={"PATH": "/usr/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    assert len(specs) == 8
    for r, (cmd, env) in enumerate(specs):
        assert cmd[0] == sys.executable and cmd[1] == os.path.join(ROOT, "bench.py") and cmd[2:] == argv
        assert (env["RANK"], env["LOCAL_RANK"], env["WORLD_SIZE"]) == (str(r), str(r), "8")
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29555"
        assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_bench_refuses_more_ranks_than_gpus():
    """--gpus N with fewer visible GPUs (none here) fails non-zero instead of
    benching fewer GPUs, unless FPF_BENCH_BACKEND=gloo asks for a rehearsal; a
    launcher's WORLD_SIZE that disagrees with --gpus fails too."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "FPF_BENCH_BACKEND")}
    env["HIP_VISIBLE_DEVICES"] = ""   # (no GPU in this container anyway; on a GPU box: none visible)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 2 and "visible" in r.stderr, r.stderr[-2000:]
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=ROOT, env=dict(env, WORLD_SIZE="4"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr, r.stderr[-2000:]


@pytest.mark.gpu
def test_bench_two_ranks_share_one_gpu():
    """`bench.py --gpus 2` exactly as the driver runs it (no launcher: bench.py
    starts its two ranks itself), over gloo so the two ranks can share the box's
    one GPU: n_gpus and the world each rank saw are 2, and the study aggregate
    covers both ranks' shards."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["FPF_BENCH_BACKEND"] = "gloo"
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1", "--no-c4", "--no-cpu-baseline",
           "--in-batches", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["rccl_world"] == 2
    agg = d["aggregate"]
    assert agg["n_scen"] == 2 * 3 * 4096 and agg["n_conv"] == agg["n_scen"]


COLLECTIVES = ("all_reduce", "all_gather", "all_gather_into_tensor", "barrier", "broadcast", "reduce",
               "reduce_scatter", "reduce_scatter_tensor", "all_to_all", "all_to_all_single", "gather", "scatter")


def _timed_rank_main(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    f = F.synthetic_feeder(30, 30)
    lo, hi = D.shard_range(rank, world, N_STUDY)
    from oracle import oracle as O
    r = O.dpf_batch(f.Dl, f.Z, F.hosting_loads(f, np.arange(lo, hi)), nthreads=2, want_full=False)
    row = torch.from_numpy(D.aggregate_results(r["status"], r["loss"], r["vmin"], r["vmax"]))
    calls = []
    saved = {n: getattr(dist, n) for n in COLLECTIVES if hasattr(dist, n)}
    for n, fn in saved.items():
        setattr(dist, n, (lambda n, fn: lambda *a, **k: (calls.append(n), fn(*a, **k))[1])(n, fn))
    try:
        elapsed, tot = D.timed_study(lambda: None, lambda: row)
    finally:
        for n, fn in saved.items():
            setattr(dist, n, fn)
    np.save(os.path.join(out_dir, f"row{rank}.npy"), row.numpy())
    np.save(os.path.join(out_dir, f"tot{rank}.npy"), tot)
    with open(os.path.join(out_dir, f"calls{rank}.txt"), "w") as fh:
        fh.write(" ".join(calls))
    dist.destroy_process_group()


def test_timed_region_has_one_collective():
    """bench.py's timed region (dist.timed_study): exactly one collective -- the
    all-gather of the per-rank aggregates -- and no barrier; every rank's study
    aggregate is fold_aggregates of the shards' rows in rank order, bit for bit."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_timed_rank_main, args=(2, _free_port(), d), nprocs=2, join=True, start_method="spawn")
        rows = [np.load(os.path.join(d, f"row{k}.npy")) for k in range(2)]
        for k in range(2):
            assert open(os.path.join(d, f"calls{k}.txt")).read().split() == ["all_gather"]
            np.testing.assert_array_equal(np.load(os.path.join(d, f"tot{k}.npy")), D.fold_aggregates(rows))
    assert D.fold_aggregates(rows)[7] == N_STUDY


def test_fold_aggregates_rank_order():
    rows = np.array([[1e16, 0.99, 1.01, 5, 0, 0, 0, 5], [1.0, 0.97, 1.02, 3, 1, 0, 1, 4],
                     [-1e16, 0.98, 1.00, 2, 0, 1, 0, 2]])
    out = D.fold_aggregates(rows)
    assert out[0] == (1e16 + 1.0) + -1e16   # sequential, in rank order (0.0 here, not 1.0)
    assert (out[1], out[2]) == (0.97, 1.02) and list(out[3:]) == [10, 1, 1, 1, 11]
    ident = D.fold_aggregates(np.zeros((0, 8)))
    assert ident[0] == 0 and ident[1] == np.inf and ident[2] == -np.inf
