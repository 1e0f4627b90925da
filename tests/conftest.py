import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs libfreedm_pf kernels)")


def pytest_collection_modifyitems(config, items):
    if any(item.get_closest_marker("gpu") for item in items):
        try:
            import torch
            has_gpu = torch.cuda.is_available()
        except Exception:
            has_gpu = False
        if not has_gpu:
            skip = pytest.mark.skip(reason="no GPU in this container (run with -m gpu on the MI355X box)")
            for item in items:
                if item.get_closest_marker("gpu"):
                    item.add_marker(skip)


def load_golden(name):
    with np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


GOLDEN_NAMES = ["g1_demo", "g1_demo_batch", "g2_dlnew", "g3_123bus", "g4_2048bus", "g5_nonconv", "g6_missing_phase"]
