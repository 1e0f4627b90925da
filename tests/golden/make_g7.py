"""G7: the VVC round on the reference's own 9-row feeder --
vvc_main's numerics (VoltVarCtrl.cpp:1141-1762) run sequentially by the C
oracle (oracle/ref_vvc.c): base loss, the gradient per phase, the step sizes'
losses, the stop index, the direction flag and the 21 S2 set-points of the
Gradient message.  Also the 123-bus synthetic feeder's round.  Run from the
repo root: `python tests/golden/make_g7.py`."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from freedm_amd import feeder as F  # noqa: E402
from freedm_amd import vvc  # noqa: E402
from oracle import oracle as O  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    for name, f in (("g7_vvc_round", F.demo_feeder()), ("g7_vvc_round_123bus", F.synthetic_feeder(123, 123))):
        r = O.vvc_main(f.Dl, f.Z)
        assert r["rc"] == 0, r["rc"]
        lens = [len(x) for x in r["g"]]
        np.savez_compressed(
            os.path.join(OUT, f"{name}.npz"), Dl=f.Dl, Z=f.Z,
            g=np.concatenate(r["g"]), load_nodes=np.concatenate(r["load_nodes"]), n_loads=np.array(lens),
            loss_fwd=r["loss_fwd"], loss_rev=r["loss_rev"], Dl_after=r["Dl"], S2=vvc.s2_setpoints(r["Dl"]),
            scalars=np.array([r[k] for k in ("ploss_orig", "vmin_orig", "vmax_orig", "c0", "stop_fwd", "stop_rev",
                                             "reversed", "sent", "ploss_after", "gmin", "gmax", "gabs_min", "calls")]))
        print(name, "stop", r["stop_fwd"], "reversed", r["reversed"], "loss", r["ploss_orig"], "->", r["ploss_after"],
              "S2[:4]", np.round(vvc.s2_setpoints(r["Dl"])[:4], 4))


if __name__ == "__main__":
    main()
