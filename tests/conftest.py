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


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_runtime_first():
    """Two HIP runtimes share a GPU test process: torch's bundled one and the ROCm one libmpcfatigue.so links.  torch's
    initialises only if it comes first (a torch tensor created after a library solve in a fresh process fails with
    "No HIP GPUs are available"), so GPU sessions initialise it before any test runs."""
    if has_gpu():
        import torch
        torch.cuda.init()
    yield


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    out = {}
    for name, N in [("G1_box_N50", 50), ("G2_box_N80", 80), ("G3_box_N80", 80), ("G4_box_N80", 80)]:
        out[name] = (np.loadtxt(os.path.join(GOLDEN, f"{name}_solution.csv"), delimiter=","), N)
    return out
