import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def has_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    out = {}
    for name, N in [("G1_box_N50", 50), ("G2_box_N80", 80), ("G3_box_N80", 80), ("G4_box_N80", 80)]:
        out[name] = (np.loadtxt(os.path.join(GOLDEN, f"{name}_solution.csv"), delimiter=","), N)
    return out
