"""One HIP runtime per process.  torch bundles its own libamdhip64 under the soname
libamdhip64.so.7 that libmpcfatigue.so links; mpc_fatigue_amd._lib.lib() maps torch's first, so the library and torch
share one runtime whichever of the two a program uses first.  Each order runs in a fresh interpreter."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

LIB_THEN_TORCH = r"""
import sys, numpy as np
sys.path.insert(0, ROOT)
from mpc_fatigue_amd import _lib, problems as PR
from mpc_fatigue_amd.gocp import GOCP
sp = PR.pilz6_bench(N=8)
r = GOCP(sp).solve(x0=np.asarray(sp["q0"])[None], init_zero=True, filter=True, bound_relax=1e-8, max_iter=3000)
assert int(r.status[0]) == 0, r.status
import torch
x = torch.arange(8, dtype=torch.float64, device="cuda")
assert float((x * 2).sum().item()) == 56.0
assert len(_lib._hip_runtimes()) == 1, _lib._hip_runtimes()
print("ok", _lib._hip_runtimes())
"""

TORCH_THEN_LIB = r"""
import sys, numpy as np
sys.path.insert(0, ROOT)
import torch
x = torch.ones(4, dtype=torch.float64, device="cuda")
from mpc_fatigue_amd import _lib, problems as PR
from mpc_fatigue_amd.gocp import GOCP
sp = PR.pilz6_bench(N=8)
g = GOCP(sp)
dev = torch.device("cuda", 0)
out = {"w": torch.empty((1, g.wsize), dtype=torch.float64, device=dev),
       "status": torch.empty(1, dtype=torch.int32, device=dev), "iters": torch.empty(1, dtype=torch.int32, device=dev),
       "kkt": torch.empty(1, dtype=torch.float64, device=dev), "obj": torch.empty(1, dtype=torch.float64, device=dev)}
q0 = torch.tensor(np.asarray(sp["q0"])[None], dtype=torch.float64, device=dev)
st = torch.cuda.Stream(dev)
g.solve_dev(q0.data_ptr(), None, None, None, 1, {k: v.data_ptr() for k, v in out.items()}, stream=st.cuda_stream,
            init_zero=True, filter=True, bound_relax=1e-8, max_iter=3000)
st.synchronize()
assert int(out["status"][0].item()) == 0
assert float(x.sum().item()) == 4.0
assert len(_lib._hip_runtimes()) == 1, _lib._hip_runtimes()
print("ok", _lib._hip_runtimes())
"""


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["library_then_torch", "torch_then_library"])
def test_one_hip_runtime_either_order(order):
    code = (LIB_THEN_TORCH if order == "library_then_torch" else TORCH_THEN_LIB).replace("ROOT", repr(ROOT))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=110)
    print(p.stdout[-2000:], p.stderr[-2000:])
    assert p.returncode == 0, p.stderr[-2000:]
    assert "ok" in p.stdout
