"""The config-1 host-synchronous VVC round (fpf_vvc_round) on the demo and
Dl_new feeders, timed as bench.py's config1_vvc_round leg (best of 20), for a
rocprofv3 kernel + copy trace of where a round's time goes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401  (the device, as in bench.py)
    from freedm_amd import PowerFlow, demo_feeder, dl_new_feeder
    for name, d in [("demo", demo_feeder()), ("dl_new", dl_new_feeder())]:
        pf = PowerFlow(d, device=0)
        for _ in range(2):
            pf.vvc_round(d.Dl)
        tt = []
        for _ in range(20):
            t0 = time.perf_counter()
            r = pf.vvc_round(d.Dl)
            tt.append(time.perf_counter() - t0)
        print(f"{name}: best {min(tt) * 1e3:.3f} ms, median {sorted(tt)[10] * 1e3:.3f} ms, stop_fwd {int(r['stop_fwd'])}, "
              f"reversed {int(r['reversed'])}", flush=True)
        pf.close()


if __name__ == "__main__":
    main()
