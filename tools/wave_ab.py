"""A/B of wave-kernel variants selected by environment variables, in one process.

    python tools/wave_ab.py "base:-" "g48:FPF_WAVE_GEOM=4,8" ... [--configs 2,4] [--reps 2]

Each variant is NAME:ENV=val+ENV2=val ("-" = none); the variables are set
before the feeder is created (the wave plan reads them there).  Per config the
launch time is the HIP-event average over back-to-back launches on one device
batch (config 2: 4096 x 123-bus scenario-fastest, 12 rotating batches; config
4: 131072 hosting scenarios, scenario-major; config 3: 2048-bus x 65536,
scenario-major).  Every variant's iterations must equal the first variant's and
V must agree to 1e-10 relative, else the run fails.
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--configs", default="2,4")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--nodes", type=int, default=0, help="feeder size override for configs 2/4")
    args = ap.parse_args()
    import torch
    from freedm_amd import PowerFlow, hosting_loads, scenario_loads, synthetic_feeder
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    cfgs = [int(c) for c in args.configs.split(",")]
    data = {}
    for c in cfgs:
        if c == 2:
            f = synthetic_feeder(args.nodes or 123, args.nodes or 123)
            B, lay = 4096, 0
            pqs = [torch.from_numpy(scenario_loads(f, np.arange(b * B, (b + 1) * B), seed=4096)).to(dev) for b in range(12)]
        elif c == 4:
            f = synthetic_feeder(args.nodes or 123, args.nodes or 123)
            B, lay = 131072, 1
            x = torch.empty((6, f.nl, B), dtype=torch.float64, device=dev)
            for a in range(0, B, 16384):
                x[:, :, a:a + 16384] = torch.from_numpy(hosting_loads(f, np.arange(a, a + 16384), seed=1 << 20)).to(dev)
            pqs = [x.permute(2, 0, 1).contiguous()]
            del x
        else:
            f = synthetic_feeder(2048, 2048)
            B, lay = 65536, 1
            base = torch.from_numpy(scenario_loads(f, np.arange(1024), seed=65536)).to(dev)
            ids = torch.arange(B, device=dev)
            x = base[:, :, ids % 1024] * (0.9 + 0.2 * ((ids * 2654435761) % 1000).double() / 1000.0)
            pqs = [x.permute(2, 0, 1).contiguous()]
            del x, base
        data[c] = (f, B, lay, pqs)
    ref = {}
    results = {}
    for rep in range(args.reps):
        for v in args.variants:
            name, envs = v.split(":", 1)
            saved = {}
            if envs != "-":
                for kv in envs.split("+"):
                    k, val = kv.split("=", 1)
                    saved[k] = os.environ.get(k)
                    os.environ[k] = val
            line = []
            for c in cfgs:
                f, B, lay, pqs = data[c]
                pf = PowerFlow(f, device=0, layout=lay, no_guard=int(os.environ.get("AB_NO_GUARD", "0")))
                pf.reserve(B)
                sh = (B, 3, pf.nn) if lay == 1 else (3, pf.nn, B)
                out = {"iters": torch.zeros(B, dtype=torch.int32, device=dev),
                       "status": torch.zeros(B, dtype=torch.int8, device=dev),
                       "loss": torch.zeros(B, dtype=torch.float64, device=dev),
                       "vmin": torch.zeros(B, dtype=torch.float64, device=dev),
                       "vmax": torch.zeros(B, dtype=torch.float64, device=dev),
                       "v_re": torch.zeros(sh, dtype=torch.float64, device=dev),
                       "v_im": torch.zeros(sh, dtype=torch.float64, device=dev)}
                solves = [pf.bind_device(p, out, stream=stream)[0] for p in pqs]
                for i in range(3):
                    solves[i % len(solves)]()
                torch.cuda.synchronize(dev)
                steps = args.steps if c != 3 else max(3, args.steps // 5)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for i in range(steps):
                    solves[i % len(solves)]()
                e1.record(stream)
                torch.cuda.synchronize(dev)
                ms = e0.elapsed_time(e1) / steps
                # correctness against the first variant (last batch solved)
                solves[(steps - 1) % len(solves)]()
                torch.cuda.synchronize(dev)
                it = out["iters"].cpu().numpy()
                V = (out["v_re"] + 1j * out["v_im"]).cpu().numpy()
                if c not in ref:
                    ref[c] = (it, V)
                    err = 0.0
                else:
                    it0, V0 = ref[c]
                    if not (it == it0).all():
                        print(f"FAIL {name} c{c}: iterations differ in {(it != it0).sum()} scenarios", flush=True)
                        sys.exit(1)
                    err = float(np.max(np.abs(V - V0) / np.maximum(np.abs(V0), 1e-300)))
                    if err > 1e-10:
                        print(f"FAIL {name} c{c}: V rel err {err:.3e}", flush=True)
                        sys.exit(1)
                results.setdefault((name, c), []).append(ms)
                line.append(f"c{c} {ms * 1e3:9.2f} us (sweeps {it.mean():.2f}, dV {err:.1e})")
                pf.close()
                del out, solves
            for k, val in saved.items():
                if val is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = val
            print(f"{name:12s} " + " | ".join(line), flush=True)
    print("best of reps:")
    for v in args.variants:
        name = v.split(":", 1)[0]
        print(f"{name:12s} " + " | ".join(f"c{c} {min(results[(name, c)]) * 1e3:9.2f} us" for c in cfgs), flush=True)


if __name__ == "__main__":
    main()
