"""Kernel time of one-scenario (and 32-scenario) device solves of the config-1
feeders, full outputs (Vpolar / PQb / PQL) against light ones (V and scalars):
HIP events around 200 back-to-back launches on one stream."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from freedm_amd import PowerFlow, demo_feeder, dl_new_feeder
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    for name, f in [("demo", demo_feeder()), ("dl_new", dl_new_feeder())]:
        pf = PowerFlow(f, device=0)
        for B in (1, 32):
            pq = torch.from_numpy(np.ascontiguousarray(np.repeat(f.Dl[:, 6:12].T[:, :, None], B, axis=2))).to(dev)
            line = []
            for full in (True, False):
                out = {"iters": torch.zeros(B, dtype=torch.int32, device=dev),
                       "status": torch.zeros(B, dtype=torch.int8, device=dev),
                       "loss": torch.zeros(B, dtype=torch.float64, device=dev),
                       "vmin": torch.zeros(B, dtype=torch.float64, device=dev),
                       "vmax": torch.zeros(B, dtype=torch.float64, device=dev),
                       "v_re": torch.zeros((3, pf.nn, B), dtype=torch.float64, device=dev),
                       "v_im": torch.zeros((3, pf.nn, B), dtype=torch.float64, device=dev)}
                if full:
                    for k in ("vpolar", "pqb", "pql"):
                        out[k] = torch.zeros((6, pf.nn, B), dtype=torch.float64, device=dev)
                solve = pf.bind_device(pq, out, stream=st)[0]
                for _ in range(10):
                    solve()
                torch.cuda.synchronize(dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(200):
                    solve()
                e1.record(st)
                torch.cuda.synchronize(dev)
                line.append(f"{'full' if full else 'light'} {e0.elapsed_time(e1) / 200 * 1e3:.1f} us")
            print(f"{name} B={B}: " + ", ".join(line), flush=True)
        pf.close()


if __name__ == "__main__":
    main()
