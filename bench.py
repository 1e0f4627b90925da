"""Benchmark: converged power-flow scenarios/s on the 123-bus feeder (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W]

N > 1: bench.py starts N rank processes itself (one per GPU, RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in their environment) before
anything touches a device, and exits with their status; under a launcher
(python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N) the
ranks come from the launcher's environment instead.

Workload = BASELINE config 2: synthetic 123-bus feeder (seed 123), a batch of
4096 seeded load/DER scenarios per GPU (weak scaling; scenario ids are global,
rank r solves ids [r*4096, (r+1)*4096)).  One step = one pass of the hot path
over that batch: one launch of libfreedm_pf's DPF kernel (the wave kernel in
the default fast mode: all sweeps, V, per-scenario loss / Vmin / Vmax /
iterations), inputs resident in HBM, per-scenario results kept for every
step.  The K steps go round robin onto two HIP streams (--streams): the
batches are independent, so a launch starts on the CUs its predecessor's last
workgroups free instead of waiting for the whole grid to drain (a 4096-scenario
launch is one round of workgroups; measured 109 -> 125 M scenarios/s,
profiles/r05c3).  After the K timed steps the study aggregate over all K x 4096 results
is reduced once on each GPU (deterministic) and combined across GPUs by one
RCCL all-gather folded in rank order (the only collective of the path and of
the timed region: freedm_amd/dist.py timed_study); each rank reads its clock
right after it, and the max over ranks is taken outside the region.
value = converged scenarios of all ranks / max-over-ranks wall time.

Also reported: the roofline of the dominant kernel (algorithmic bytes per
SURVEY.md 8(d) / one launch's HIP-event time: with two streams the K launches
are re-run back to back on one stream after the timed region for it, so that it
is the kernel's own duration, as a rocprofv3 trace of --streams 1 reports it;
the timed region's GPU time per launch is `kernel_ms_timed_region`), and the CPU
oracle (oracle/ref_dpf.c, a scalar port) timed on the host's cores on a bounded
sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6        # MI355X fp64 vector peak
SCEN_PER_GPU = 4096
FEEDER_NODES, FEEDER_SEED, SCEN_SEED = 123, 123, 4096
# BASELINE.json configs measurable on one GPU: (nodes, feeder seed, scenarios per GPU,
# scenario seed, load model).  Config 2 is the bench line; 3 and 4 are diagnostics
# (--config 3|4) for the roofline at throughput-sized batches.
CONFIGS = {2: (123, 123, 4096, 4096, "scenario"),
           3: (2048, 2048, 65536, 65536, "scenario"),
           4: (123, 123, 131072, 1 << 20, "hosting")}
# batch layout each config is benched in (fpf_opts.layout; --layout overrides)
# (measured, profiles/r02e_layout: config 3 17.5 -> 9.9 ms per launch and
# config 4 1.14 -> 1.06 ms with [B][6][Nl]; config 2 39.4 vs 41.0 us then; since the
# table-driven scenario-major staging, profiles/r04f: config 2 38.6-39.1 vs 40.6-41.1 us)
LAYOUT = {2: 1, 3: 1, 4: 1}


def bytes_alg_per_scenario(nb: int, nn: int) -> int:
    """S in (48 B per branch) + V out (48 B per node) + iters,
    loss, Vmin, Vmax (28 B); state-resident model (state stays in LDS)."""
    return 48 * nb + 48 * nn + 28


def bytes_alg_streaming(nb: int, nn: int, k_sum: float, n_scen: int) -> float:
    """SURVEY.md 8(d) config 3 (Nb = 2047): the per-scenario state cannot stay
    on chip, so each sweep also moves V and Ib once each way (192 B per branch
    per sweep) on top of the compulsory bytes."""
    return bytes_alg_per_scenario(nb, nn) * n_scen + 192.0 * nb * k_sum


def usable_cpus() -> tuple[int, dict]:
    """CPUs this process can actually run on: the affinity mask, capped by the
    cgroup CPU quota (cpu.max) -- on the GPU box the affinity mask lists all 256
    host threads while the quota grants 16 CPUs of time, so more threads than
    the quota only time-slice."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    n = aff if quota is None else max(1, min(aff, int(quota)))
    return n, {"affinity": aff, "cgroup_quota_cpus": quota, "nproc_host": os.cpu_count()}


def _host_cores():
    """(physical cores, logical CPUs) of the host from /proc/cpuinfo."""
    phys, logical = set(), 0
    try:
        pid = core = None
        for line in open("/proc/cpuinfo"):
            if line.startswith("processor"):
                logical += 1
            elif line.startswith("physical id"):
                pid = line.split(":")[1].strip()
            elif line.startswith("core id"):
                core = line.split(":")[1].strip()
                phys.add((pid, core))
    except OSError:
        pass
    return len(phys) or None, logical or None


def _time_oracle(O, feeder, pq, threads: int, seconds: float):
    n_conv = passes = 0
    t0 = time.perf_counter()
    while True:
        r = O.dpf_batch(feeder.Dl, feeder.Z, pq, nthreads=threads, want_full=False)
        n_conv += int((r["status"] == 0).sum())
        passes += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return n_conv / dt, passes, dt


def cpu_baseline(feeder, seconds: float = 10.0, chunk: int = 32768, config1: bool = True, legs: int = 3,
                 gpu_solve=None, n_check: int = 256):
    """The CPU oracle (oracle/ref_dpf.c, a scalar port of DPF_return7 + the VVC
    reductions) on this host: on every usable CPU (value, cores) and on one CPU,
    each as the median of `legs` legs of seconds / legs over the same chunk of the
    config-2 batch.  The single-CPU legs run with the process pinned to one CPU
    of its affinity set (os.sched_setaffinity), so the lone thread is not moved
    between cores; the per-core rate is the better of that and the all-CPU rate
    divided by its threads, and the full-host estimate scales it by the host's
    physical cores (not measured: the box's cgroup grants only `cores` CPUs)."""
    from oracle import oracle as O
    from freedm_amd import scenario_loads
    threads, cpu_info = usable_cpus()
    pq = scenario_loads(feeder, np.arange(chunk), seed=SCEN_SEED)
    leg_s = max(1.0, seconds / legs)
    all_legs = [_time_oracle(O, feeder, pq, threads, leg_s) for _ in range(legs)]
    v_all = float(np.median([r[0] for r in all_legs]))
    passes, dt = sum(r[1] for r in all_legs), sum(r[2] for r in all_legs)
    aff = sorted(os.sched_getaffinity(0))
    try:
        os.sched_setaffinity(0, {aff[len(aff) // 2]})
        one_legs = [_time_oracle(O, feeder, pq, 1, leg_s) for _ in range(legs)]
    finally:
        os.sched_setaffinity(0, set(aff))
    v_one = float(np.median([r[0] for r in one_legs]))
    passes1, dt1 = sum(r[1] for r in one_legs), sum(r[2] for r in one_legs)
    per_core = max(v_one, v_all / threads)
    phys, logical = _host_cores()
    out_c1 = None
    if config1:
        out_c1 = config1_cpu()
    out = {"value": v_all, "unit": "converged scenarios/s", "cores": threads, "kind": "port",
           "sample": f"median of {legs} legs, {passes} passes x {chunk} scenarios of the batch ({feeder.name}, seed "
                     f"{SCEN_SEED}), oracle/ref_dpf.c ({threads} pthreads, -O3, no FMA), {dt:.1f} s; single core: "
                     f"median of {legs} legs pinned to CPU {aff[len(aff) // 2]}, {passes1} passes x {chunk} "
                     f"scenarios, {dt1:.1f} s",
           "legs": [r[0] for r in all_legs],
           "single_core": {"value": v_one, "unit": "converged scenarios/s", "cores": 1,
                           "legs": [r[0] for r in one_legs]},
           "parallel_efficiency": v_all / (v_one * threads),
           "per_core_rate": per_core,
           "cpu_model": _cpu_model(), "host_physical_cores": phys, "host_logical_cpus": logical,
           }
    if out_c1:
        out["config1_vvc_main"] = out_c1
    out.update(cpu_info)
    if phys:
        # not measured: what the whole host would give if the port scaled linearly
        # over every physical core at the better-measured per-core rate
        out["full_host_linear_estimate"] = per_core * phys
    if gpu_solve is not None:
        # the benched kernel against this oracle on the first n_check scenarios of the
        # sample (the parity bar: V within 1e-10 relative, identical sweep counts)
        sub = np.ascontiguousarray(pq[:, :, :n_check])
        c = O.dpf_batch(feeder.Dl, feeder.Z, sub, nthreads=threads)
        gv = gpu_solve(sub)
        a = gv["V_re"] + 1j * gv["V_im"]
        b = c["V_re"] + 1j * c["V_im"]
        out["parity_sample"] = {"scenarios": int(sub.shape[2]),
                                "max_v_rel_err": float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300))),
                                "iters_identical": bool((gv["iters"] == c["iters"]).all()),
                                "mean_sweeps": float(c["iters"].mean()),
                                "note": "the benched kernel vs oracle/ref_dpf.c on the first scenarios of the "
                                        "CPU-baseline sample (same feeder and scenario generator)"}
    return out


def _gpu_solve_scen_fastest(pf, pq):
    """pf.solve on a [6][Nl][B] host batch, results [..][B] whatever pf's layout."""
    if pf.opts.layout == 1:
        r = pf.solve(np.ascontiguousarray(pq.transpose(2, 0, 1)), full=True)
        return {"V_re": np.moveaxis(r["V_re"], 0, -1), "V_im": np.moveaxis(r["V_im"], 0, -1), "iters": r["iters"]}
    return pf.solve(pq, full=True)


def multi_leg(n_vis: int) -> dict:
    """The one-process multi-GPU entry a Broker would use (fpf_multi_*: one host
    thread drives every visible GPU; VoltVarCtrl.cpp:1141 runs on the Broker's
    single io_service thread): the config-4 hosting study (131 072 scenarios,
    host buffers, scalars out) on 1 and on all n_vis visible devices."""
    from freedm_amd import MultiPowerFlow, hosting_loads, synthetic_feeder
    feeder = synthetic_feeder(CONFIGS[4][0], CONFIGS[4][1])
    Bm = CONFIGS[4][2]
    pq_m = np.empty((Bm, 6, feeder.nl))
    for a in range(0, Bm, 16384):
        pq_m[a:a + 16384] = hosting_loads(feeder, np.arange(a, a + 16384), seed=CONFIGS[4][3]).transpose(2, 0, 1)
    mres = {}
    for n_dev in sorted({1, n_vis}):
        mp = MultiPowerFlow(feeder, n_gpus=n_dev, layout=1)
        rm = mp.solve(pq_m, full=False)
        tm = []
        for _ in range(3):
            t0 = time.perf_counter()
            rm = mp.solve(pq_m, full=False)
            tm.append(time.perf_counter() - t0)
        mres[str(n_dev)] = {"ms": min(tm) * 1e3, "scen_per_s": Bm / min(tm),
                            "converged": int(rm["aggregate"]["n_conv"]), "n_scen": int(rm["aggregate"]["n_scen"])}
        mp.close()
    return {"workload": f"BASELINE config 4 study, {Bm} hosting scenarios, host buffers (843 MB in, scalars out), "
                        "fpf_multi_solve", "devices": mres,
            "speedup_all_vs_1": mres["1"]["ms"] / mres[str(n_vis)]["ms"],
            "note": "PCIe-bound (host-resident inputs); never the bench value"}


def _multi_leg_child(n_vis: int, timeout_s: float = 240.0) -> dict:
    """multi_leg() in a child process (python bench.py --multi-leg N) with a time
    limit: fpf_multi over several GPUs runs only where a process sees them (the
    driver's 8-GPU node), so a failure there is reported, not fatal to the line."""
    import subprocess
    try:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--multi-leg", str(n_vis)],
                           capture_output=True, text=True, timeout=timeout_s)
        lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if r.returncode == 0 and lines:
            return json.loads(lines[-1])
        return {"error": f"child exit {r.returncode}", "stderr_tail": r.stderr[-600:]}
    except subprocess.TimeoutExpired:
        return {"error": f"timed out after {timeout_s:.0f} s"}


def config1_feeders():
    """BASELINE config 1's feeders: the reference's own 9-row demo feeder
    (load_system_data.cpp), Broker/Dl_new.mat (IEEE 34-node, with the supplied Z)
    and the synthetic 123-bus feeder."""
    from freedm_amd import demo_feeder, dl_new_feeder, synthetic_feeder
    return [("demo", demo_feeder()), ("dl_new", dl_new_feeder()), ("123bus", synthetic_feeder(123, 123))]


def config1_cpu(reps: int = 5):
    """One sequential vvc_main round of the reference (gradient + step-size
    search, 2m+1 DPF calls; oracle/ref_vvc.c, VoltVarCtrl.cpp:1141-1762) per
    config-1 feeder, one core, best of `reps`."""
    from oracle import oracle as O
    out = {}
    for name, f in config1_feeders():
        O.vvc_main(f.Dl, f.Z)
        t_round = []
        for _ in range(reps):
            t0 = time.perf_counter()
            r = O.vvc_main(f.Dl, f.Z)
            t_round.append(time.perf_counter() - t0)
        out[name] = {"ms": min(t_round) * 1e3, "dpf_calls": int(r["calls"]), "stop_fwd": int(r["stop_fwd"]),
                     "reversed": int(r["reversed"])}
    out["note"] = "oracle/ref_vvc.c vvc_main (VoltVarCtrl.cpp:1141-1762), best of %d, one core" % reps
    return out


def round_scenarios(f, B: int, seed: int = 11, lo: float = 0.6, hi: float = 1.4) -> np.ndarray:
    """B load scenarios ([6][Nl][B]) of a control table that keep its (int) load
    tests (fpf_vvc_gradient_batch shares the load lists): entries whose test would
    flip keep the control's value (tests/test_vvc_round.py)."""
    base = np.ascontiguousarray(f.Dl[:, 6:12].T)[:, :, None]
    pq = base * np.random.default_rng(seed).uniform(lo, hi, size=(6, f.nl, B))
    flip = (pq.astype(np.int64) != 0) != (base.astype(np.int64) != 0)
    return np.ascontiguousarray(np.where(flip, base, pq))


def vvc_batch_leg(local: int, B: int = 64, cpu_sample: int = 8) -> dict:
    """BASELINE config 1 as a Monte Carlo over loads: B whole VVC rounds
    (fpf_vvc_round_batch: batched gradients, every scenario's 101 step sizes in
    one batch, the reversed searches in another) per config-1 feeder, beside the
    oracle's sequential vvc_main (VoltVarCtrl.cpp:1141-1762) on a sample of the
    same scenarios, one core."""
    from freedm_amd import PowerFlow
    from oracle import oracle as O
    out = {}
    for name, f in config1_feeders():
        pq = round_scenarios(f, B)
        pf = PowerFlow(f, device=local)
        r = pf.vvc_round_batch(f.Dl, pq)
        tt = []
        for _ in range(3):
            t0 = time.perf_counter()
            r = pf.vvc_round_batch(f.Dl, pq)
            tt.append(time.perf_counter() - t0)
        pf.close()
        ts = []
        agree = 0
        for s in range(cpu_sample):
            D = f.Dl.copy()
            D[:, 6:12] = pq[:, :, s].T
            t0 = time.perf_counter()
            o = O.vvc_main(D, f.Z)
            ts.append(time.perf_counter() - t0)
            # a round the reference throws on (a step solve that does not converge,
            # rc != 0) agrees when the batch flags it (tests/test_vvc_round.py)
            if o["rc"] != 0:
                agree += int(r["nonconv"][s] == 1)
            else:
                agree += int(r["nonconv"][s] == 0 and
                             all(int(r[k][s]) == int(o[k]) for k in ("stop_fwd", "stop_rev", "reversed", "sent")))
        cpu_round_ms = float(np.median(ts)) * 1e3
        out[name] = {"rounds": B, "gpu_ms": min(tt) * 1e3, "gpu_rounds_per_s": B / min(tt),
                     "cpu_round_ms": cpu_round_ms, "cpu_rounds_per_s_one_core": 1e3 / cpu_round_ms,
                     "speedup_vs_one_core": (B / min(tt)) / (1e3 / cpu_round_ms),
                     "reversed": int(np.sum(r["reversed"])), "n_bad": int(r["n_bad"]),
                     "decisions_equal_oracle": f"{agree}/{cpu_sample}"}
    out["note"] = ("fpf_vvc_round_batch, host buffers, best of 3; CPU: oracle/ref_vvc.c vvc_main per scenario "
                   "(median of a sample), one core; tests/test_vvc_round.py checks every scenario's decisions")
    return out


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _pmc_traffic(workload: str, kernel: str | None = None, key: str = "hbm_bytes_per_launch"):
    """Per-launch HBM bytes of the dominant kernel for `workload` ("123-bus x
    4096") from the committed rocprofv3 --pmc summaries
    (profiles/pmc_traffic.json, tools/pmc_summary.py), or None: the guide's
    correction, 2 x FETCH_SIZE + WRITE_SIZE."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p))
        e = d.get("by_workload", {}).get(workload)
        if e is None and d.get("workload") == workload:
            e = d
        if e and kernel and e.get("kernel") != kernel:
            return None   # measured on another kernel
        return e.get(key) if e else None
    except (OSError, ValueError, AttributeError):
        return None


def _instruction_efficiency(workload: str, kernel: str, flops_per_launch: float) -> dict:
    """Useful fp64 flops per launch (the flop model above) / the issued VALU lane
    capacity of the launch, 2 flops (an FMA) x 64 lanes per wave64 VALU
    instruction, from the committed SQ_INSTS_VALU pass of this workload
    (profiles/pmc_traffic.json "valu_insts_per_launch", tools/runs/gpu_pmc_sq.sh): how
    much of what the kernel issues on the VALU is the path's arithmetic (the rest:
    DPP moves, address and loop arithmetic, the rounds of the scans)."""
    v = _pmc_traffic(workload, kernel, key="valu_insts_per_launch")
    if not v:
        return {}
    return {"valu_insts_per_launch": v, "instruction_efficiency": flops_per_launch / (128.0 * v),
            "valu_source": _pmc_traffic(workload, kernel, key="valu_tag")}


def _loads_on_device(torch, dev, loads, feeder, ids, seed, chunk=8192, layout=0):
    """[6][Nl][len(ids)] scenario loads of the global ids, generated on the host
    in chunks, scenario-fastest on the device."""
    out = torch.empty((6, feeder.nl, len(ids)), dtype=torch.float64, device=dev)
    for a in range(0, len(ids), chunk):
        b = min(len(ids), a + chunk)
        out[:, :, a:b] = torch.from_numpy(loads(feeder, ids[a:b], seed=seed)).to(dev)
    # FPF_LAYOUT_SCEN_MAJOR: [B][6][Nl], one scenario per contiguous block
    return out if layout == 0 else out.permute(2, 0, 1).contiguous()


def _copy_bandwidth(torch, dev, nbytes=1 << 30, reps=10):
    """Device-to-device copy rate (read + write bytes / s) of a 1 GiB buffer:
    the achievable-HBM reference the roofline's 8 TB/s spec is checked against."""
    a = torch.empty(nbytes // 8, dtype=torch.float64, device=dev).fill_(1.0)
    b = torch.empty_like(a)
    for _ in range(2):
        b.copy_(a)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize(dev)
    gbs = 2 * nbytes * reps / (e0.elapsed_time(e1) / 1e3) / 1e9
    del a, b
    return gbs


def _wave_kernel_name(nb: int) -> str:
    """The fast-mode kernel of a feeder of nb branches: the per-wavefront wave
    kernel (<= 256), the wave-block kernel (257..2048), the paired wave-block
    kernel (2049..4096; fpf_wcoop.hip)."""
    return "dpf_wave_kernel" if nb <= 256 else ("dpf_wblk_kernel" if nb <= 2048 else "dpf_wcoop_kernel")


def _diag_4096(torch, local, stream, dev):
    """Diagnostic leg: a 4096-bus synthetic feeder x 16 384 scenarios (scenario
    major, 512 seeded scenarios x a per-scenario load multiplier) on the paired
    wave-block kernel, beside the exact generic kernel on the same device inputs
    (the only other kernel that solves feeders of more than 2048 branches):
    launch times, the state-resident roofline fraction, and the fast kernel's
    agreement with the exact one (iteration counts, max V relative difference)."""
    from freedm_amd import PowerFlow, scenario_loads, synthetic_feeder
    f = synthetic_feeder(4096, 4096)
    B = 16384
    base = torch.from_numpy(scenario_loads(f, np.arange(512), seed=16384)).to(dev)
    ids = torch.arange(B, device=dev)
    mult = 0.9 + 0.2 * ((ids * 2654435761) % 1000).double() / 1000.0
    d = (base[:, :, ids % 512] * mult).permute(2, 0, 1).contiguous()
    del base
    out = {}
    for name, exact in (("fast", 0), ("exact", 1)):
        pf = PowerFlow(f, device=local, exact=exact, layout=1)
        pf.reserve(B)
        ms, o = _kernel_ms(torch, pf, d, B, 3, 1, stream, dev)
        out[name] = (ms, o, pf.kernel, pf.info["nb"], pf.nn)
        pf.close()
    (msf, of, kf, nb, nn), (mse, oe, ke, _, _) = out["fast"], out["exact"]
    a = of["v_re"] + 1j * of["v_im"]
    b = oe["v_re"] + 1j * oe["v_im"]
    vrel = float(((a - b).abs() / b.abs()).max().item())
    del a, b
    bpa = bytes_alg_per_scenario(nb, nn)
    conv = int((of["status"] == 0).sum().item())
    return {"workload": f"diagnostic: {nn}-bus synthetic feeder, {B} scenarios per launch (scenario major)",
            "kernel": _wave_kernel_name(nb) if kf == "wave" else kf, "kernel_ms": msf,
            "converged_scenarios_per_s": conv / (msf / 1e3),
            "roofline_frac": bpa * B / (msf / 1e3) / 1e9 / HBM_PEAK_GBS, "bytes_alg_per_scenario": bpa,
            "mean_sweeps": float(of["iters"].double().mean().item()),
            "exact_kernel": ke, "exact_kernel_ms": mse, "speedup_vs_exact": mse / msf,
            "iters_equal_exact": bool(torch.equal(of["iters"], oe["iters"])),
            "status_equal_exact": bool(torch.equal(of["status"], oe["status"])),
            "max_v_rel_diff_vs_exact": vrel,
            "note": "tests/test_gpu_wcoop.py checks the same batch against the oracle (strided sample) and the "
                    "exact kernel (every scenario)"}


def _shuffled_units(f, seed):
    """The feeder with its [separator + lateral block] units in a seeded order
    (tests/lag_tables.py: laterals listed before their taps' rows -- tables the
    tree plan declines, DPF_return7.cpp:134-195 solves them in row order)."""
    from freedm_amd import Feeder
    Dl = np.asarray(f.Dl)
    cut = [0] + [i for i in range(Dl.shape[0]) if Dl[i, 0] == 0] + [Dl.shape[0]]
    units = [Dl[cut[i]:cut[i + 1]] for i in range(1, len(cut) - 1)]
    order = np.random.default_rng(seed).permutation(len(units))
    return Feeder(np.vstack([Dl[:cut[1]]] + [units[i] for i in order]), f.Z, name=f"{f.name}-shuffled{seed}")


def _zeroed_units(f):
    """Phase c zeroed (a two-phase line code, no phase-c load) on every second
    lateral unit that no other unit taps (tests/lag_tables.py: zeroed)."""
    from freedm_amd import Feeder
    Dl = np.array(f.Dl, copy=True)
    Z = np.vstack([f.Z, np.diag([f.Z[0, 0], f.Z[1, 1], 0])])
    code = Z.shape[0] // 3
    sep = [i for i in range(Dl.shape[0]) if Dl[i, 0] == 0] + [Dl.shape[0]]
    taps = {int(Dl[i + 1, 1]) for i in sep[:-1] if i + 1 < Dl.shape[0]}
    leaves = [u for u in range(len(sep) - 1) if not any(int(Dl[r, 2]) in taps for r in range(sep[u] + 1, sep[u + 1]))]
    for u in leaves[::2]:
        Dl[sep[u] + 1:sep[u + 1], 3] = code
        Dl[sep[u] + 1:sep[u + 1], 10:12] = 0.0
    return Feeder(Dl, Z, name=f"{f.name}-zeroed")


def _diag_sequential_order(torch, local, stream, dev):
    """Diagnostic leg: feeders whose lateral units are listed in a shuffled order
    (the sequential-order plan, DESIGN 5.0e: the fast kernels' FULL variant; one
    with zeroed phases too) at 4096 scenarios (scenario major), beside the exact
    generic kernel -- until
    round 5 the only kernel for such tables -- and the tree-ordered feeder's own
    fast solve of the same loads: launch times, identical iteration counts and
    status, max V relative difference."""
    from freedm_amd import PowerFlow, scenario_loads, synthetic_feeder
    out = {}
    for name, n, seed in (("123bus_shuffled", 123, 1), ("123bus_shuffled_zeroed", 123, 1), ("2048bus_shuffled", 2048, 13)):
        f0 = synthetic_feeder(n, n)
        if name.endswith("_zeroed"):
            f0 = _zeroed_units(f0)
        f = _shuffled_units(f0, seed)
        B = 4096
        pq = scenario_loads(f, np.arange(B), seed=B + 11)
        d = torch.from_numpy(np.ascontiguousarray(pq.transpose(2, 0, 1))).to(dev)
        legs = {}
        for kind, exact in (("fast", 0), ("exact", 1)):
            pf = PowerFlow(f, device=local, exact=exact, layout=1)
            pf.reserve(B)
            ms, o = _kernel_ms(torch, pf, d, B, 3, 1, stream, dev)
            legs[kind] = (ms, o, pf.kernel, pf.info["nb"], pf.nn)
            pf.close()
        (msf, of, kf, nb, nn), (mse, oe, ke, _, _) = legs["fast"], legs["exact"]
        conv = oe["status"] == 0
        a = torch.complex(of["v_re"], of["v_im"])
        b = torch.complex(oe["v_re"], oe["v_im"])
        # (zeroed phases: V exactly 0 in both)
        r = torch.where(conv.view(-1, 1, 1) & (b.abs() > 0), (a - b).abs() / b.abs().clamp_min(1e-300),
                        torch.zeros_like(b.real))
        vrel = float(r.max().item())
        del a, b, r, d
        zz = ", phase c zeroed on every second leaf unit" if name.endswith("_zeroed") else ""
        out[name] = {"workload": f"{nn}-bus synthetic feeder{zz}, lateral units shuffled (seed {seed}), {B} scenarios",
                     "kernel": _wave_kernel_name(nb) if kf == "wave" else kf, "variant": "full (sequential order)",
                     "kernel_ms": msf, "converged_scenarios_per_s": int(conv.sum().item()) / (msf / 1e3),
                     "mean_sweeps": float(of["iters"].double().mean().item()),
                     "exact_kernel": ke, "exact_kernel_ms": mse, "speedup_vs_exact": mse / msf,
                     "iters_equal_exact": bool(torch.equal(of["iters"], oe["iters"])),
                     "status_equal_exact": bool(torch.equal(of["status"], oe["status"])),
                     "max_v_rel_diff_vs_exact": vrel,
                     "note": "tests/test_gpu_lag.py checks these tables against the oracle"}
        del of, oe
    return out


def _diag_heavy(torch, local, stream, dev):
    """Diagnostic leg: the config-2 and config-3 feeders at their full batch sizes
    under heavier, mixed loads (each scenario's loads scaled by a factor spread
    over 1.5 .. 3.0: 6 .. 12 sweeps instead of the calibrated batches' 5), on the
    fast kernels, beside the exact generic kernel on the same device inputs:
    launch times, mean sweeps, identical iteration counts and status, max V
    relative difference (the parity margin at full size)."""
    from freedm_amd import PowerFlow, scenario_loads, synthetic_feeder
    out = {}
    for name, n, B, lay in (("config2_heavy", 123, 4096, 0), ("config3_heavy", 2048, 65536, 1)):
        f = synthetic_feeder(n, n)
        NB = min(B, 1024)
        base = torch.from_numpy(scenario_loads(f, np.arange(NB), seed=B + 7)).to(dev)
        ids = torch.arange(B, device=dev)
        mult = 1.5 * torch.pow(torch.tensor(2.0, dtype=torch.float64, device=dev),
                               ((ids * 2654435761) % 1000).double() / 999.0)   # 1.5 .. 3.0
        d = base[:, :, ids % NB] * mult
        if lay == 1:
            d = d.permute(2, 0, 1).contiguous()
        del base
        legs = {}
        for kind, exact in (("fast", 0), ("exact", 1)):
            pf = PowerFlow(f, device=local, exact=exact, layout=lay)
            pf.reserve(B)
            ms, o = _kernel_ms(torch, pf, d, B, 3, 1, stream, dev)
            legs[kind] = (ms, o, pf.kernel, pf.info["nb"], pf.nn)
            pf.close()
        (msf, of, kf, nb, nn), (mse, oe, ke, _, _) = legs["fast"], legs["exact"]
        conv = oe["status"] == 0
        vrel = 0.0
        for c0 in range(0, B, 4096):   # (in scenario chunks: the 2048-bus V is 6.4 GB per part)
            sl = (slice(c0, c0 + 4096),) if lay == 1 else (slice(None), slice(None), slice(c0, c0 + 4096))
            a = torch.complex(of["v_re"][sl], of["v_im"][sl])
            b = torch.complex(oe["v_re"][sl], oe["v_im"][sl])
            cc = conv[c0:c0 + 4096]
            cm = cc.view(-1, 1, 1) if lay == 1 else cc.view(1, 1, -1)
            r = torch.where(cm, (a - b).abs() / b.abs(), torch.zeros_like(b.real))
            vrel = max(vrel, float(r.max().item()))
            del a, b, r
        del d
        bpa = bytes_alg_per_scenario(nb, nn)
        it = of["iters"].double()
        out[name] = {"workload": f"{nn}-bus synthetic feeder x {B} scenarios, loads x 1.5 .. 3.0",
                     "kernel": _wave_kernel_name(nb) if kf == "wave" else kf, "kernel_ms": msf,
                     "converged_scenarios_per_s": int(conv.sum().item()) / (msf / 1e3),
                     "roofline_frac": bpa * B / (msf / 1e3) / 1e9 / HBM_PEAK_GBS,
                     "mean_sweeps": float(it.mean().item()), "min_sweeps": int(it.min().item()),
                     "max_sweeps": int(it.max().item()), "vmin": float(of["vmin"][conv].min().item()),
                     "exact_kernel": ke, "exact_kernel_ms": mse,
                     "iters_equal_exact": bool(torch.equal(of["iters"], oe["iters"])),
                     "status_equal_exact": bool(torch.equal(of["status"], oe["status"])),
                     "max_v_rel_diff_vs_exact": vrel}
        del of, oe
    return out


def _kernel_ms(torch, pf, d_pq, B, steps, warmup, stream, dev, want_v=True):
    """Average launch time (HIP events on the launch stream) of `steps`
    back-to-back solves of the device batch d_pq, plus the iterations."""
    out = {"iters": torch.zeros(B, dtype=torch.int32, device=dev), "status": torch.zeros(B, dtype=torch.int8, device=dev),
           "loss": torch.zeros(B, dtype=torch.float64, device=dev), "vmin": torch.zeros(B, dtype=torch.float64, device=dev),
           "vmax": torch.zeros(B, dtype=torch.float64, device=dev)}
    if want_v:
        sh = (B, 3, pf.nn) if pf.opts.layout == 1 else (3, pf.nn, B)
        out.update(v_re=torch.zeros(sh, dtype=torch.float64, device=dev),
                   v_im=torch.zeros(sh, dtype=torch.float64, device=dev))
    solve = pf.bind_device(d_pq, out, stream=stream)[0]
    for _ in range(warmup):
        solve()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        solve()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) / steps, out


def rank_launch_specs(n: int, argv: list, port: int, base_env: dict | None = None) -> list:
    """(command, environment) of each of the n rank processes `bench.py --gpus n`
    starts when no launcher set WORLD_SIZE: the same script and arguments, one
    rank per GPU (LOCAL_RANK r -> cuda:r), rendezvous on 127.0.0.1:port."""
    env0 = dict(os.environ if base_env is None else base_env)
    specs = []
    for r in range(n):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        specs.append(([sys.executable, os.path.abspath(__file__)] + list(argv), env))
    return specs


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list) -> int:
    """Start the n rank processes (rank_launch_specs) and wait for them; if one
    fails the others are stopped (they would wait at a barrier).  Returns the
    first non-zero exit status, else 0.  Called before this process imports
    anything that initialises a GPU (device_count does not, on this image)."""
    import subprocess
    import torch
    n_vis = torch.cuda.device_count()
    gloo = os.environ.get("FPF_BENCH_BACKEND", "nccl") == "gloo"
    if n > n_vis and not gloo:
        print(f"bench.py: --gpus {n} but {n_vis} GPU(s) visible (FPF_BENCH_BACKEND=gloo rehearses more ranks "
              "than GPUs on shared devices)", file=sys.stderr, flush=True)
        return 2
    procs = [subprocess.Popen(cmd, env=env) for cmd, env in rank_launch_specs(n, argv, _free_port())]
    rc = 0
    try:
        while procs:
            for p in list(procs):
                c = p.poll()
                if c is None:
                    continue
                procs.remove(p)
                if c != 0 and rc == 0:
                    rc = c
                    for q in procs:
                        q.terminate()
            time.sleep(0.05)
    finally:
        for q in procs:
            q.kill()
    return rc


def _wave_rtc_builds():
    """per-plan hipRTC wave kernels built in this process (fpf_opts.specialize:
    the wave launches of >= 4096 scenarios run them, FPF_WAVE_RTC overrides;
    fpf_rtc.cpp: WAVE_RTC_DEFAULT_MIN)"""
    import ctypes
    from freedm_amd import _lib
    L = _lib.load()
    L.fpf_wave_rtc_builds.restype = ctypes.c_int
    return int(L.fpf_wave_rtc_builds())


def main():
    if len(sys.argv) == 3 and sys.argv[1] == "--multi-leg":   # (bench.py's own child, _multi_leg_child)
        print(json.dumps(multi_leg(int(sys.argv[2]))), flush=True)
        return
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS),
                    help="BASELINE config: 2 (the bench line), 3 (2048-bus x 65536), 4 (hosting study shard)")
    ap.add_argument("--scenarios", type=int, default=0, help="scenarios per GPU per step (0: the config's)")
    ap.add_argument("--nodes", type=int, default=0, help="diagnostic: synthetic feeder size override (seed = nodes)")
    ap.add_argument("--kernel", default="auto")
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--no-specialize", action="store_true")
    ap.add_argument("--exact", type=int, default=0, help="1: the reference's roundings (bit-identical mode)")
    ap.add_argument("--no-guard", action="store_true", help="diagnostic: fast mode without the convergence guard")
    ap.add_argument("--layout", type=int, default=-1,
                    help="batch layout: 0 [6][Nl][B] (scenario fastest), 1 [B][6][Nl] (scenario major); "
                         "-1: the config's default (LAYOUT)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-v-out", action="store_true", help="diagnostic: do not request the V outputs")
    ap.add_argument("--in-batches", type=int, default=0,
                    help="distinct input batches the steps cycle through (0: enough for > 256 MiB of inputs, so "
                         "the Infinity Cache cannot hold them; 1: re-solve one batch)")
    ap.add_argument("--no-c4", action="store_true", help="skip the config-4 throughput leg of the config-2 run")
    ap.add_argument("--streams", type=int, default=2,
                    help="launch the steps round robin on this many HIP streams (independent batches; "
                         "measured: 2 beats 1 and 4, profiles/r05st)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU, started here before any device is touched
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        print(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} from the launcher but --gpus {args.gpus}",
              file=sys.stderr, flush=True)
        sys.exit(2)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU (RCCL over xGMI).  FPF_BENCH_BACKEND=gloo with more ranks
    # than GPUs rehearses the multi-rank path on a one-GPU box (ranks share it)
    backend = os.environ.get("FPF_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from freedm_amd import PowerFlow, hosting_loads, scenario_loads, synthetic_feeder

    n_nodes, f_seed, b_cfg, s_seed, model = CONFIGS[args.config]
    if args.nodes:
        n_nodes, f_seed = args.nodes, args.nodes
    loads = {"scenario": scenario_loads, "hosting": hosting_loads}[model]
    feeder = synthetic_feeder(n_nodes, f_seed)
    layout = LAYOUT[args.config] if args.layout < 0 else args.layout
    pf = PowerFlow(feeder, device=local, kernel=args.kernel, tile=args.tile, specialize=not args.no_specialize,
                   exact=args.exact, layout=layout, no_guard=int(args.no_guard))
    B = args.scenarios or b_cfg
    pf.reserve(B)
    from freedm_amd import dist as D
    # the steps cycle through n_in distinct input batches (together more than the
    # 256 MiB Infinity Cache, so every step streams its loads from HBM); weak
    # scaling: rank r's batch b holds global ids (b * world + r) * B ... + B
    batch_bytes = 48 * feeder.nl * B
    n_in = args.in_batches or max(1, min(64, -(-300 * 2 ** 20 // batch_bytes)))
    n_in = min(n_in, max(args.steps, 1))
    d_pqs = []
    for b in range(n_in):
        lo, hi = D.shard_range(rank, world, world * B)
        ids = np.arange(lo, hi) + b * world * B
        d_pqs.append(_loads_on_device(torch, dev, loads, feeder, ids, s_seed, layout=layout))
    # per-scenario outputs of every timed step (the study's results); V is
    # overwritten step after step
    K = max(args.steps, 1)
    res = {"iters": torch.zeros((K, B), dtype=torch.int32, device=dev),
           "status": torch.zeros((K, B), dtype=torch.int8, device=dev),
           "loss": torch.zeros((K, B), dtype=torch.float64, device=dev),
           "vmin": torch.zeros((K, B), dtype=torch.float64, device=dev),
           "vmax": torch.zeros((K, B), dtype=torch.float64, device=dev)}
    vsh = (B, 3, pf.nn) if layout == 1 else (3, pf.nn, B)
    v_out = {} if args.no_v_out else {"v_re": torch.zeros(vsh, dtype=torch.float64, device=dev),
                                      "v_im": torch.zeros(vsh, dtype=torch.float64, device=dev)}
    stream = torch.cuda.current_stream(dev)
    # --streams S: step i on stream i % S (stream 0 = the current one), each
    # stream with its own V buffer; the batches are independent, so a launch
    # can start on the CUs the previous one's last workgroups free
    S = max(1, args.streams)
    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
    v_outs = [v_out] + [{k: torch.zeros_like(v) for k, v in v_out.items()} for _ in range(S - 1)]
    solves = [pf.bind_device(d_pqs[i % n_in], dict(v_outs[i % S], **{k: t[i] for k, t in res.items()}),
                             stream=streams[i % S])[0]
              for i in range(K)]
    flat = {k: t.view(-1) for k, t in res.items()}
    agg = torch.zeros(8, dtype=torch.float64, device=dev)

    def step(i):
        # one batch: the DPF kernel -- all sweeps, V, loss / Vmin / Vmax / iterations
        # per scenario
        solves[i]()

    study_agg = pf.bind_aggregate(flat, agg, n_scen=K * B, stream=stream)
    host_rows = torch.zeros(8 * world, dtype=torch.float64, pin_memory=True)

    def study_aggregate():
        # once per study: [loss_sum, vmin, vmax, n_conv, n_nonconv, n_over, n_under,
        # n_scen] over every scenario solved (deterministic reduction)
        study_agg()
        return agg

    for i in range(args.warmup):
        step(i % K)
    study_aggregate()
    torch.cuda.synchronize(dev)
    conv_per_step = int((res["status"][0] == 0).sum().item())

    # HIP events on the launch stream bracket the K back-to-back launches of the
    # timed region: average kernel time = their elapsed time / K
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_submit = 0.0
    joins = [torch.cuda.Event() for _ in streams[1:]]

    # the start event of the timed region's GPU-time diagnostic (ev0 -> ev1,
    # roofline.kernel_ms_timed_region) and the side streams' waits on it are
    # recorded just before the clock starts (then synchronised), not inside the
    # region: instrumentation, not the workload -- inside, the event and the
    # cross-stream waits held the first launches back, 127.7-131.1 vs 132.4-136.2 M
    # scenarios/s at the driver's K = 20 (profiles/r06s2_ev0*; FPF_BENCH_EV0_OUT=0
    # restores the old placement, 2 records the event inside without the waits)
    ev0_mode = os.environ.get("FPF_BENCH_EV0_OUT", "1")
    ev0_out = ev0_mode == "1"

    def mark_start():
        ev0.record(stream)
        if ev0_mode != "2":
            for st in streams[1:]:
                st.wait_event(ev0)

    def run_steps():
        nonlocal t_submit
        t = time.perf_counter()
        if not ev0_out:
            mark_start()
        for i in range(args.steps):
            step(i)
        for st, e in zip(streams[1:], joins):
            e.record(st)
            stream.wait_event(e)
        ev1.record(stream)
        t_submit = time.perf_counter() - t

    # the timed region: the K solves, the study aggregate and the one collective
    # (an all-gather of the per-GPU aggregates over RCCL/xGMI, folded in rank
    # order); each rank reads its clock without a further barrier
    sync = lambda: torch.cuda.synchronize(dev)   # noqa: E731
    # (the region's host path once untimed -- aggregate, the collective, the copy
    # and the fold -- so that the timed one runs warm)
    D.timed_study(lambda: None, study_aggregate, sync=sync, host=host_rows)
    if world > 1:
        dist.barrier()
    if ev0_out:
        mark_start()
    sync()
    elapsed, tot = D.timed_study(run_steps, study_aggregate, sync=sync, host=host_rows)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # the GPU time per launch in the timed region (with S > 1 streams the launches
    # overlap: a launch starts on the CUs the previous one's last workgroups free)
    pipe_kern_s = ev0.elapsed_time(ev1) / args.steps / 1e3
    avg_kern_s = pipe_kern_s
    if S > 1:
        # the roofline is the kernel's: one launch's own duration, the same K
        # launches back to back on one stream after the timed region (what a
        # rocprofv3 kernel trace of `--streams 1` reports per launch)
        serial = [pf.bind_device(d_pqs[i % n_in], dict(v_out, **{k: t[i] for k, t in res.items()}), stream=stream)[0]
                  for i in range(K)]
        torch.cuda.synchronize(dev)
        ev0.record(stream)
        for i in range(args.steps):
            serial[i]()
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        avg_kern_s = ev0.elapsed_time(ev1) / args.steps / 1e3
    n_conv_all = float(tot[3])
    value = n_conv_all / elapsed
    nb, nn = pf.info["nb"], pf.nn
    bpa = bytes_alg_per_scenario(nb, nn)
    k_sum = float(res["iters"][:args.steps].sum().item())
    # the dominant kernel: fast mode runs the wave kernel (<= 256 branches) or the
    # wave-block kernel (257..2048, one scenario per workgroup), both with the
    # state on chip; exact mode the tiled or the generic kernel
    kname = {"tiled": "fpf_rtc_tiled" if pf.info["specialized"] else "dpf_tiled_kernel",
             "wave": _wave_kernel_name(nb), "generic": "dpf_generic3_kernel"}[pf.kernel]
    if pf.kernel == "generic":
        # the state streams through HBM every sweep (SURVEY 8(d) config 3 model)
        bytes_launch = bytes_alg_streaming(nb, nn, k_sum / args.steps, B)
        model = "streaming (state through HBM every sweep)"
    else:
        bytes_launch = bpa * B
        model = "state-resident (loads in, V and scalars out)"
    achieved = bytes_launch / avg_kern_s / 1e9
    traffic = _pmc_traffic(f"{n_nodes}-bus x {B}", kname)
    # algorithmic fp64 flops per scenario = 123 Nb k_s + 60 Nn, over
    # the timed launches, against the 78.6 TFLOP/s fp64 vector peak
    flops = 123.0 * nb * k_sum + 60.0 * nn * B * args.steps
    fp64_tflops = flops / (avg_kern_s * args.steps) / 1e12

    if rank == 0:
        res = {
            "metric": "converged power-flow scenarios/sec, %d-bus feeder" % n_nodes,
            "value": value,
            "unit": "scenarios/s",
            "n_gpus": world,
            "rccl_world": dist.get_world_size() if world > 1 else 1,
            "backend": backend if world > 1 else None,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64 (complex fp64)",
            "data": f"synthetic (seeded {n_nodes}-bus radial feeder + seeded {model} load/PV scenarios)",
            "config": {"workload": f"BASELINE config {args.config}: {n_nodes}-bus feeder, {B} scenarios per GPU per step",
                       "feeder": feeder.name, "scenarios_per_gpu": B, "kernel": pf.kernel,
                       "input_batches": n_in, "input_mib": n_in * batch_bytes / 2 ** 20,
                       "tile": pf.info["tile"], "specialized": pf.info["specialized"],
                       "wave_rtc_builds": _wave_rtc_builds(), "exact": bool(args.exact),
                       "layout": ["[6][Nl][B] scenario fastest", "[B][6][Nl] scenario major"][layout],
                       "parallelism": f"scenario shards x{world}", "streams": S},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kname, "model": model,
                         "bytes_alg_per_scenario": bytes_launch / B, "kernel_ms": avg_kern_s * 1e3,
                         "kernel_ms_timed_region": pipe_kern_s * 1e3,
                         "fp64": {"achieved": fp64_tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                                  "frac": fp64_tflops / FP64_PEAK_TFLOPS,
                                  "mean_sweeps": k_sum / (B * args.steps),
                                  **_instruction_efficiency(f"{n_nodes}-bus x {B}", kname,
                                                            flops / args.steps)}},
            "aggregate": {"loss_sum_kw": float(tot[0]), "vmin": float(tot[1]), "vmax": float(tot[2]),
                          "n_conv": int(tot[3]), "n_nonconv": int(tot[4]), "n_over": int(tot[5]),
                          "n_under": int(tot[6]), "n_scen": int(tot[7])},
            "converged_per_step_rank0": conv_per_step,
            "host_submit_ms_per_step": t_submit / args.steps * 1e3,
        }
        if world == 1 and args.config == 2 and not args.no_c4 and not args.nodes and not args.scenarios:
            # the throughput-sized roofline next to the bench line (BASELINE config 4:
            # one GPU's 131 072-scenario shard of the hosting study, 843 MB of inputs)
            n4, s4, b4, seed4, m4 = CONFIGS[4]
            ids4 = np.arange(b4)
            lay4 = LAYOUT[4] if args.layout < 0 else args.layout
            pf4 = PowerFlow(feeder, device=local, kernel=args.kernel, exact=args.exact, layout=lay4)
            d4 = _loads_on_device(torch, dev, hosting_loads, feeder, ids4, seed4, layout=lay4)
            pf4.reserve(b4)
            ms4, o4 = _kernel_ms(torch, pf4, d4, b4, 10, 3, stream, dev)
            conv4 = int((o4["status"] == 0).sum().item())
            ach4 = bpa * b4 / (ms4 / 1e3) / 1e9
            res["roofline_config4"] = {
                "workload": f"BASELINE config 4: {n4}-bus feeder, {b4} hosting scenarios per GPU per launch",
                "bound": "hbm", "achieved": ach4, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach4 / HBM_PEAK_GBS,
                "traffic": _pmc_traffic(f"{n4}-bus x {b4}"),
                "kernel_ms": ms4, "bytes_alg_per_scenario": bpa,
                "converged_scenarios_per_s": conv4 / (ms4 / 1e3),
                "layout": ["[6][Nl][B] scenario fastest", "[B][6][Nl] scenario major"][lay4],
                "mean_sweeps": float(o4["iters"].double().mean().item()),
                **_instruction_efficiency(f"{n4}-bus x {b4}", "dpf_wave_kernel",
                                          123.0 * pf4.info["nb"] * float(o4["iters"].double().sum().item())
                                          + 60.0 * pf4.nn * b4)}
            del d4
            pf4.close()
            # BASELINE config 3 beside it: the 2048-bus feeder x 65 536 scenarios on
            # the wave-block kernel (scenario-major), 1024 seeded scenarios x a
            # per-scenario load multiplier so all 65 536 differ (tests/test_gpu_wblk.py);
            # `python bench.py --config 3` generates every scenario and adds its CPU leg
            n3, s3f, b3, seed3, _ = CONFIGS[3]
            f3 = synthetic_feeder(n3, s3f)
            pf3 = PowerFlow(f3, device=local, kernel=args.kernel, exact=args.exact, layout=LAYOUT[3])
            base3 = torch.from_numpy(scenario_loads(f3, np.arange(1024), seed=seed3)).to(dev)
            ids3 = torch.arange(b3, device=dev)
            mult3 = 0.9 + 0.2 * ((ids3 * 2654435761) % 1000).double() / 1000.0
            d3 = base3[:, :, ids3 % 1024] * mult3
            if LAYOUT[3] == 1:
                d3 = d3.permute(2, 0, 1).contiguous()
            del base3
            pf3.reserve(b3)
            ms3, o3 = _kernel_ms(torch, pf3, d3, b3, 3, 1, stream, dev)
            conv3 = int((o3["status"] == 0).sum().item())
            bpa3 = bytes_alg_per_scenario(pf3.info["nb"], pf3.nn)
            ach3 = bpa3 * b3 / (ms3 / 1e3) / 1e9
            k3 = "dpf_wblk_kernel" if pf3.kernel == "wave" else {"generic": "dpf_generic3_kernel"}.get(pf3.kernel, pf3.kernel)
            res["roofline_config3"] = {
                "workload": f"BASELINE config 3: {n3}-bus feeder, {b3} scenarios per GPU per launch",
                "bound": "hbm", "achieved": ach3, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach3 / HBM_PEAK_GBS,
                "traffic": _pmc_traffic(f"{n3}-bus x {b3}", k3), "kernel": k3,
                "model": "state-resident (loads in, V and scalars out)" if pf3.kernel == "wave" else
                         "state-resident bytes; this kernel streams its state (see --config 3)", "kernel_ms": ms3,
                "bytes_alg_per_scenario": bpa3, "converged_scenarios_per_s": conv3 / (ms3 / 1e3),
                "mean_sweeps": float(o3["iters"].double().mean().item()),
                "layout": ["[6][Nl][B] scenario fastest", "[B][6][Nl] scenario major"][LAYOUT[3]],
                # SURVEY 8(d) priced config 3 with its state streaming through HBM
                # (2.16 MB per scenario at 5 sweeps: 3.70 M scen/s at 100 % of 8 TB/s);
                # this kernel keeps the state on chip, so that rate is exceeded
                "survey_streaming_roofline_scen_per_s": HBM_PEAK_GBS * 1e9 / (
                    bytes_alg_streaming(pf3.info["nb"], pf3.nn, float(o3["iters"].double().mean().item()), 1)),
                "vs_survey_streaming_roofline": (conv3 / (ms3 / 1e3)) / (HBM_PEAK_GBS * 1e9 / bytes_alg_streaming(
                    pf3.info["nb"], pf3.nn, float(o3["iters"].double().mean().item()), 1))}
            del d3, o3
            pf3.close()
            # feeders of 2049..4096 branches: the paired wave-block kernel
            res["diag_4096bus"] = _diag_4096(torch, local, stream, dev)
            # the calibrated batches run 5 sweeps each: the same feeders under heavier,
            # mixed loads at full size, with the parity margin against the exact kernel
            res["diag_heavy"] = _diag_heavy(torch, local, stream, dev)
            # tables whose rows do not follow the feeder tree (the sequential-order plan)
            res["diag_sequential_order"] = _diag_sequential_order(torch, local, stream, dev)
            copy = _copy_bandwidth(torch, dev)
            res["hbm_copy_check"] = {"device_copy_gbs": copy, "spec_gbs": HBM_PEAK_GBS,
                                     "copy_frac_of_spec": copy / HBM_PEAK_GBS,
                                     "config2_frac_of_copy": achieved / copy,
                                     "config4_frac_of_copy": ach4 / copy,
                                     "note": "torch copy_ of 1 GiB, read+write bytes; roofline.frac stays "
                                             "against the 8 TB/s spec"}
        if world == 1 and args.config == 2 and not args.no_c4 and not args.nodes and not args.scenarios:
            # BASELINE config 1: one whole VVC round (fpf_vvc_round: the gradient
            # after a device solve, all m_max+1 step sizes as one batch, the
            # reversal) per config-1 feeder (demo, Dl_new.mat, 123-bus);
            # host-synchronous, best of 20 (5 for the 123-bus feeder)
            c1 = {}
            for name1, d1 in config1_feeders():
                pf1 = PowerFlow(d1, device=local)
                for _ in range(2):
                    r1 = pf1.vvc_round(d1.Dl)
                tt = []
                for _ in range(5 if d1.nl > 100 else 20):
                    t0 = time.perf_counter()
                    r1 = pf1.vvc_round(d1.Dl)
                    tt.append(time.perf_counter() - t0)
                c1[name1] = {"gpu_ms": min(tt) * 1e3, "stop_fwd": int(r1["stop_fwd"]), "sent": int(r1["sent"]),
                             "reversed": int(r1["reversed"]), "kernel": pf1.kernel, "nl": int(d1.nl)}
                pf1.close()
            # the host-buffer entry (fpf_solve_batch: PCIe copies in and out included;
            # per-scenario scalars out, no V), one config-2 batch
            pq_h = d_pqs[0].cpu().numpy()
            pf.solve(pq_h, full=False)
            th = []
            for _ in range(5):
                t0 = time.perf_counter()
                rh = pf.solve(pq_h, full=False)
                th.append(time.perf_counter() - t0)
            res["host_buffer_path"] = {"scen_per_s": int((rh["status"] == 0).sum()) / min(th),
                                       "ms_per_batch": min(th) * 1e3,
                                       "note": "fpf_solve_batch with host buffers (26 MB H2D, scalars D2H), "
                                               "best of 5; never the bench value"}
            # BASELINE config 5: the multi-area solve (fpf_areas_*) of the 123-bus
            # feeder cut into 3 areas, one config-2 batch, host buffers, tolerance
            # 1e-12, beside the monolithic host-buffer solve of the same batch
            from freedm_amd import AreaPowerFlow
            from freedm_amd.feeder import subtree_node_areas
            pq_a = pq_h if layout == 0 else np.ascontiguousarray(pq_h.transpose(1, 2, 0))   # areas: [6][Nl][B]
            ap = AreaPowerFlow(feeder, subtree_node_areas(feeder, [30, 60]), device=local)
            ra = ap.solve(pq_a, tol=1e-12, v_out=False)
            ta, tv = [], []
            for _ in range(5):   # scalars out, as the monolithic host-buffer solve above
                t0 = time.perf_counter()
                ra = ap.solve(pq_a, tol=1e-12, v_out=False)
                ta.append(time.perf_counter() - t0)
            for _ in range(3):   # and with V back (24 MB)
                t0 = time.perf_counter()
                ap.solve(pq_a, tol=1e-12)
                tv.append(time.perf_counter() - t0)
            res["config5_areas"] = {"areas": len(ap.area_nodes), "area_nodes": ap.area_nodes, "scenarios": int(B),
                                    "ms_per_batch": min(ta) * 1e3, "ms_per_batch_with_v": min(tv) * 1e3,
                                    "outer_iterations": int(ra["iters"].max()),
                                    "converged": int((ra["status"] == 0).sum()),
                                    "monolithic_host_ms": min(th) * 1e3,
                                    "vs_monolithic": min(ta) / min(th),
                                    "note": "fpf_areas_solve, host buffers (scalars out, as the monolithic figure; "
                                            "with_v: V back too), boundary exchange to 1e-12 p.u., device-side stop "
                                            "test; tests/test_areas.py checks V against the monolithic solve to 1e-10"}
            ap.close()
            # the one-process multi-GPU entry a Broker would use (fpf_multi_*: one host
            # thread drives every visible GPU, VoltVarCtrl.cpp:1141 runs on the Broker's
            # single io_service thread): the config-4 hosting study (131 072 scenarios,
            # host buffers, scalars out) over n = 1 and all visible devices.  Only when
            # more than one GPU is visible to this process (FPF_BENCH_MULTI=1 forces it
            # on one GPU to exercise the leg)
            n_vis = torch.cuda.device_count()
            if (n_vis > 1 and os.environ.get("FPF_BENCH_MULTI") != "0") or os.environ.get("FPF_BENCH_MULTI") == "1":
                # in a child process with a time limit: the bench line does not depend on it
                res["multi_gpu_inproc"] = _multi_leg_child(n_vis)
            c1["note"] =("fpf_vvc_round (gradient + the step sizes batched (the first 32, the rest only without a stop) + reversal), host-synchronous, "
                          "per config-1 feeder")
            res["config1_vvc_round"] = c1
            if not args.no_cpu_baseline:
                res["config1_vvc_round_batch"] = vvc_batch_leg(local)
        if world == 1 and args.config == 3 and not args.no_cpu_baseline and not args.nodes:
            # the 2048-bus feeder on the host: a bounded sample of 1024 scenarios
            cb = cpu_baseline(feeder, seconds=args.cpu_seconds, chunk=1024, config1=False,
                              gpu_solve=lambda x: _gpu_solve_scen_fastest(pf, x))
            res["cpu_baseline"] = cb
            res["speedup_vs_cpu"] = value / cb["value"]
            res["speedup_vs_cpu_single_core"] = value / cb["single_core"]["value"]
        if world == 1 and args.config == 2 and not args.no_cpu_baseline:
            cb = cpu_baseline(feeder, seconds=args.cpu_seconds, gpu_solve=lambda x: _gpu_solve_scen_fastest(pf, x))
            if "config1_vvc_round" in res and "config1_vvc_main" in cb:
                for name1, c in res["config1_vvc_round"].items():
                    if isinstance(c, dict) and name1 in cb["config1_vvc_main"]:
                        c["cpu_ms"] = cb["config1_vvc_main"][name1]["ms"]
                        c["cpu_dpf_calls"] = cb["config1_vvc_main"][name1]["dpf_calls"]
                        c["speedup"] = c["cpu_ms"] / c["gpu_ms"]
            res["cpu_baseline"] = cb
            res["speedup_vs_cpu"] = value / cb["value"]
            res["speedup_vs_cpu_single_core"] = value / cb["single_core"]["value"]
            if cb.get("full_host_linear_estimate"):
                res["speedup_vs_cpu_full_host_estimate"] = value / cb["full_host_linear_estimate"]
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
