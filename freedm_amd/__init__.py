"""freedm_amd -- MI355X-native batched distribution power flow for the FREEDM
DGI Broker's Volt-VAR Control solve (reference: Broker/src/vvc/DPF_return7.cpp).

The product is libfreedm_pf (C ABI, include/freedm_pf.h; gfx950 HIP kernels in
freedm_amd/csrc/).  This package is its host-side mirror for Python callers:
feeder data (feeder.py), the batched solver and the DPF_return7 drop-in
(engine.py).
"""
from .feeder import (Feeder, demo_feeder, dl_new_feeder, synthetic_feeder, scenario_loads,
                     hosting_loads, load_raw_ascii, load_arma_bin, save_arma_bin, save_raw_ascii)

__all__ = ["Feeder", "demo_feeder", "dl_new_feeder", "synthetic_feeder", "scenario_loads", "hosting_loads",
           "load_raw_ascii", "load_arma_bin", "save_arma_bin", "save_raw_ascii",
           "PowerFlow", "MultiPowerFlow", "AreaPowerFlow", "DPF_return7", "VPQ", "DPFError", "NonConvergedError", "build"]


def __getattr__(name):
    # the engine loads libfreedm_pf (and torch's HIP runtime) lazily
    if name in ("PowerFlow", "MultiPowerFlow", "AreaPowerFlow", "DPF_return7", "VPQ", "DPFError", "NonConvergedError"):
        from . import engine
        return getattr(engine, name)
    raise AttributeError(name)


def build(verbose: bool = False) -> str:
    """Compile libfreedm_pf for gfx950 in-tree (freedm_amd/lib/libfreedm_pf.so)."""
    import os
    import subprocess
    here = os.path.dirname(os.path.abspath(__file__))
    jobs = os.environ.get("MAX_JOBS", "4")
    subprocess.run(["make", "-C", os.path.join(here, "csrc"), f"-j{min(int(jobs), 16)}"] + ([] if verbose else ["-s"]),
                   check=True)
    return os.path.join(here, "lib", "libfreedm_pf.so")
